#!/bin/bash
# Round 6, the last build: r6_final_evid.sh plus the weak layouts as virtual
# ranks and the C3 / C5-size rank proxies at the default schedule.
#   bash tools/gpu/r6_final_evid2.sh COMMIT OUT
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
E=${2:-gpurun_out/r6evid}
bash tools/gpu/r6_final_evid.sh $C $E || exit 1
for b in 2x1 2x2 2x4; do
  v=$(( ${b%x*} * ${b#*x} ))
  NLH_VIRTUAL_RANKS=$v timeout -k 10 300 python bench.py --blocks $b --steps 200 --pmc off --no-cpu-baseline > $E/weak_v${v}.json 2> $E/weak_v${v}.err || exit 1
done
timeout -k 10 300 python tools/rank_proxy.py 16384 8192 200 2 0 20 26 28 > $E/c3_rank_proxy.jsonl 2> $E/c3_rank_proxy.err || exit 1
timeout -k 10 300 python tools/rank_proxy.py 4096 4096 200 2 0 4 20 26 > $E/c2_rank_proxy.jsonl 2> $E/c2_rank_proxy.err || exit 1
echo done > $E/done2
