#!/bin/bash
# Round 5: the 20-step C2 line with the host waits spinning (NLH_SYNC=0, the
# default) against HIP's auto scheduling (NLH_SYNC=3), interleaved
set -o pipefail
O=gpurun_out/r5sync
mkdir -p $O
for i in 1 2 3; do
  for m in 0 3; do
    NLH_SYNC=$m timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --pmc off > $O/bench20_sync${m}_$i.json 2> $O/bench20_sync${m}_$i.err || exit 1
  done
done
echo done > $O/done
