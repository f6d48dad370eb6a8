#!/bin/bash
# Round 6: k_prefix_rt / k_prefix_rtc output rows per work item R
# (NLH_PREFIX_ROWS): the prefix parity tests at the R values given, then bench
# lines interleaved per horizon.
#   bash tools/gpu/r6_prefix_rows.sh OUT "RTEST..." "R..." "EPS LATTICE STEPS" ...
#   (R = 0: the library's choice by eps)
set -o pipefail
export TMPDIR=/tmp
O=$1; RT=$2; RS=$3; shift 3
mkdir -p $O
for R in $RT; do
  NLH_PREFIX_ROWS=$R timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stable_dt.py tests/test_gpu_parity.py -k "prefix or huge or knob or unsupported" > $O/pytest_r$R.log 2>&1 || exit 1
  tail -1 $O/pytest_r$R.log
done
for rep in 1 2; do
for spec in "$@"; do
  read -r e n k <<< "$spec"
  for R in $RS; do
    NLH_PREFIX_ROWS=$R timeout -k 10 300 python bench.py --eps $e --lattice $n --steps $k --warmup 1 --warmup-ms 0 --pmc off --no-cpu-baseline > $O/e${e}_r${R}_$rep.json 2> $O/e${e}_r${R}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/e${e}_r${R}_$rep.json')); print($e, $R, $rep, round(d['value'],4), round(d['ms_per_step'],3))"
  done
done
done
echo done > $O/done
