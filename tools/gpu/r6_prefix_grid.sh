#!/bin/bash
# Round 6: chunked prefix kernel, waves per workgroup W x output rows R
# (NLH_PREFIX_WAVES, NLH_PREFIX_ROWS) per horizon, bench lines interleaved.
#   bash tools/gpu/r6_prefix_grid.sh OUT "W:R ..." "EPS LATTICE STEPS" ...
set -o pipefail
export TMPDIR=/tmp
O=$1; WR=$2; shift 2
mkdir -p $O
for rep in 1 2; do
for spec in "$@"; do
  read -r e n k <<< "$spec"
  for wr in $WR; do
    W=${wr%:*}; R=${wr#*:}
    NLH_PREFIX_WAVES=$W NLH_PREFIX_ROWS=$R timeout -k 10 300 python bench.py --eps $e --lattice $n --steps $k --warmup 1 --warmup-ms 0 --pmc off --no-cpu-baseline > $O/e${e}_w${W}_r${R}_$rep.json 2> $O/e${e}_w${W}_r${R}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('$O/e${e}_w${W}_r${R}_$rep.json')); print($e, $W, $R, $rep, round(d['value'],4), round(d['ms_per_step'],3))"
  done
done
done
echo done > $O/done
