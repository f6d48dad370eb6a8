#!/bin/bash
# Round 5: the driver-form 20-step C2 line with HIP's kernel-argument segment
# forced into device memory (HIP_FORCE_DEV_KERNARG=1) or host memory (=0)
# against the runtime default, interleaved, three runs each; and the same
# over 200 steps (the fixed launch/sync cost diluted)
#   bash tools/gpu/r5_kernarg.sh -> gpurun_out/r5ka/
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5ka
mkdir -p $O
for i in 1 2 3; do
  for v in def 1 0; do
    if [ $v = def ]; then
      timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --pmc off > $O/b20_${v}_$i.json 2> $O/b20_${v}_$i.err || exit 1
    else
      HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --pmc off > $O/b20_${v}_$i.json 2> $O/b20_${v}_$i.err || exit 1
    fi
  done
done
echo done > $O/done
