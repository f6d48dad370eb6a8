#!/bin/bash
# Round 6: k_prefix_rtc (W = 1) vs k_prefix_rtw (W = 2, 4, 8 waves sharing one
# staged prefix row; NLH_PREFIX_WAVES): the chunked-kernel parity tests at each
# forced W, then bench lines interleaved per horizon (R by eps).
#   bash tools/gpu/r6_prefix_waves.sh OUT "WTEST..." "W..." "EPS LATTICE STEPS" ...
#   (W = 0: the library's choice by eps)
set -o pipefail
export TMPDIR=/tmp
O=$1; WT=$2; WS=$3; shift 3
mkdir -p $O
for W in $WT; do
  NLH_PREFIX_WAVES=$W timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stable_dt.py tests/test_gpu_parity.py -k "(rtc or huge or knob) and not 4832" > $O/pytest_w$W.log 2>&1 || exit 1
  tail -1 $O/pytest_w$W.log
done
for rep in 1 2; do
for spec in "$@"; do
  read -r e n k <<< "$spec"
  for W in $WS; do
    NLH_PREFIX_WAVES=$W timeout -k 10 300 python bench.py --eps $e --lattice $n --steps $k --warmup 1 --warmup-ms 0 --pmc off --no-cpu-baseline > $O/e${e}_w${W}_$rep.json 2> $O/e${e}_w${W}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/e${e}_w${W}_$rep.json')); print($e, $W, $rep, round(d['value'],4), round(d['ms_per_step'],3))"
  done
done
done
echo done > $O/done
