#!/bin/bash
# Round 6, the build the round ends on: evidence.sh part 1 (suite, smoke,
# three 20-step C2 lines), then the test-mode 20-step line, C5's uneven
# 25-tile map over 8 virtual owners and C3 as 8 virtual ranks.
#   bash tools/gpu/r6_final.sh BUILD OUT
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
O=${2:-gpurun_out/r6final}
bash tools/gpu/evidence.sh $C 1 $O $O || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --test-mode > $O/bench20_test.json 2> $O/bench20_test.err || exit 1
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --map tests/golden/reference_inputs/load_balance_25s_8n.txt --tile 9216 --steps 20 --pmc off --no-cpu-baseline > $O/c5_map.json 2> $O/c5_map.err || exit 1
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --strong --lattice 32768 --blocks 2x4 --steps 20 --pmc off --no-cpu-baseline > $O/c3_v8.json 2> $O/c3_v8.err || exit 1
echo done > $O/done2
