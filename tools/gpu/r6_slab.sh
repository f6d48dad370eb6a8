#!/bin/bash
# Round 6: weak-scaling block layouts on one GPU as virtual ranks, 4096^2 per
# rank: the 2D blocks of bench.py's default (2x1, 2x2, 2x4) against slabs
# (1x2, 1x4, 1x8: top / bottom bands only, two neighbours per rank), twice.
#   bash tools/gpu/r6_slab.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6slab}
mkdir -p $O
for round in 1 2; do
  for b in 2x1 1x2 2x2 1x4 2x4 1x8; do
    v=$(( ${b%x*} * ${b#*x} ))
    NLH_VIRTUAL_RANKS=$v timeout -k 10 300 python bench.py --blocks $b --steps 200 --pmc off --no-cpu-baseline > $O/weak_${b}_$round.json 2> $O/weak_${b}_$round.err || exit 1
    python3 -c "import json; d=json.load(open('$O/weak_${b}_$round.json')); print('$b', round(d['value'], 1), d['exchange']['exposed_share_of_pass'])"
  done
done
echo done > $O/done
