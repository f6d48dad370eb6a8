#!/bin/bash
# Round 6: a C3 strong-scaling rank (16384 x 8192 of the 2x4 layout) on one
# GPU: alone and with the exchange-path schedule forced on all four sides,
# under schedule knobs (tools/rank_proxy.py, 200 steps, two interleaved reps).
#   bash tools/gpu/r6_c3_rank.sh OUT "NAME:ENV=V,ENV=V" ...
set -o pipefail
export TMPDIR=/tmp
O=$1; shift
mkdir -p $O
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env ${envs//,/ } timeout -k 10 300 python tools/rank_proxy.py 16384 8192 200 2 0 1 > $O/$name.jsonl 2> $O/$name.err || exit 1
  python3 -c "
import json
rs=[json.loads(l) for l in open('$O/$name.jsonl')]
print('$name', ' '.join('m%d:%.0f' % (r['mask'], r['us_per_pass']) for r in rs))"
done
echo done > $O/done
