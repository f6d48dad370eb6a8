#!/bin/bash
# Round 5, call W: k_pair_split workgroups per CU the C2 segments are sized
# for (NLH_PAIR_CU 4 / 5 / 6; the kernel holds 162 VGPRs and 27.7 KB LDS:
# 5 workgroups fit a CU), 200-step and 20-step lines, interleaved
set -o pipefail
O=gpurun_out/${OUT:-r5w}
mkdir -p $O
for rep in 1 2; do
  for cu in ${CUS:-4 5 6}; do
    NLH_PAIR_CU=$cu timeout -k 10 200 python bench.py --steps 200 --pmc off --no-cpu-baseline > $O/s200_cu${cu}_$rep.json 2> $O/s200_cu${cu}_$rep.err || exit 1
    NLH_PAIR_CU=$cu timeout -k 10 200 python bench.py --steps 20 --warmup 5 --pmc off --no-cpu-baseline > $O/s20_cu${cu}_$rep.json 2> $O/s20_cu${cu}_$rep.err || exit 1
  done
done
echo done > $O/done
