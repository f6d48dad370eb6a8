#!/bin/bash
# Round 6: one rank's share of a weak-scaling pass on one GPU -- the C2 block
# alone, with the exchange-path schedule forced on all four sides
# (NLH_FORCE_BANDS: bands, events, no messages), and 4096^2 as 2x1 blocks over
# RCCL to self; 200-step lines interleaved.
#   bash tools/gpu/r6_rank_proxy.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6proxy}
mkdir -p $O
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --pmc off --no-cpu-baseline > $O/one_$rep.json 2> $O/one_$rep.err || exit 1
  NLH_FORCE_BANDS=1 timeout -k 10 120 python bench.py --steps 200 --warmup 20 --pmc off --no-cpu-baseline > $O/bands_$rep.json 2> $O/bands_$rep.err || exit 1
  NLH_RCCL_SELF=1 timeout -k 10 120 python bench.py --strong --lattice 4096 --blocks 2x1 --steps 200 --warmup 20 --pmc off --no-cpu-baseline > $O/split2_$rep.json 2> $O/split2_$rep.err || exit 1
  for v in one bands split2; do
    python3 -c "import json; d=json.load(open('$O/${v}_$rep.json')); print('$v', $rep, round(d['value'],1), round(d['ms_per_step']*2e3,1))"
  done
done
echo done > $O/done
