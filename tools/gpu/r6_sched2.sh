#!/bin/bash
# Round 6: exchange schedule NLH_SCHED 2 (bands on the exchange stream, the
# default) vs 0 (bands on a third stream): C5's uneven map and the 2x2 weak
# layout as virtual ranks, C3 / C5-size rank proxies (tools/rank_proxy.py).
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6sched2}; mkdir -p $O
for sc in 2 0 2 0; do
  NLH_SCHED=$sc NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --map tests/golden/reference_inputs/load_balance_25s_8n.txt --tile 9216 --steps 20 --pmc off --no-cpu-baseline > $O/c5_s$sc.json 2> $O/c5_s$sc.err || exit 1
  NLH_SCHED=$sc NLH_VIRTUAL_RANKS=4 timeout -k 10 300 python bench.py --blocks 2x2 --steps 200 --pmc off --no-cpu-baseline > $O/weakv4_s$sc.json 2> $O/weakv4_s$sc.err || exit 1
  for f in c5 weakv4; do python3 -c "import json; d=json.load(open('$O/${f}_s$sc.json')); print('${f}_s$sc', round(d['value'],1))"; done
done
for sc in 2 0; do
  NLH_SCHED=$sc timeout -k 10 300 python tools/rank_proxy.py 16384 8192 200 2 20 26 28 > $O/c3rank_s$sc.jsonl 2> $O/c3rank_s$sc.err || exit 1
  NLH_SCHED=$sc timeout -k 10 300 python tools/rank_proxy.py 9216 9216 100 2 0 1 26 > $O/c5tile_s$sc.jsonl 2> $O/c5tile_s$sc.err || exit 1
  python3 -c "
import json
for f in ('c3rank','c5tile'):
    rs=[json.loads(l) for l in open('$O/%s_s$sc.jsonl' % f)]
    print(f+'_s$sc', ' '.join('m%d:%.0f' % (r['mask'], r['us_per_pass']) for r in rs))"
done
echo done > $O/done
