#!/bin/bash
# Round 6: one rank's pass with the exchange-path schedule forced on all four
# sides (NLH_FORCE_BANDS: bands, events, no messages) under the schedule knobs
# (interior workgroups per CU, where the bands run, stream priority, band
# segment height); 200-step C2 lines interleaved.
#   bash tools/gpu/r6_band_sched.sh OUT "NAME:ENV=V,ENV=V ..."
set -o pipefail
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
for rep in 1 2; do
  for spec in "$@"; do
    name=${spec%%:*}; envs=${spec#*:}
    env ${envs//,/ } timeout -k 10 120 python bench.py --steps 200 --warmup 20 --pmc off --no-cpu-baseline > $O/${name}_$rep.json 2> $O/${name}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/${name}_$rep.json')); print('$name', $rep, round(d['value'],1), round(d['ms_per_step']*2e3,1))"
  done
done
echo done > $O/done
