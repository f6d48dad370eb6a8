#!/bin/bash
# Round 6, the build the round ends on: rocprofv3 / PMC evidence of the
# bench's dominant kernel (C2, C2 test mode; tools/bench_evidence.sh), eps 300
# (k_prefix_rtw), the
# test-mode 20-step line, C3 as 8 virtual ranks and C5's uneven map.
#   bash tools/gpu/r6_final_evid.sh COMMIT OUT
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
E=${2:-gpurun_out/r6evid}
mkdir -p $E
NLH_N=4096 NLH_EPS=8 tools/bench_evidence.sh $E/c2 k_pair_split weak_4096_eps8_prod 33554432 $C -- || exit 1
NLH_N=4096 NLH_EPS=8 NLH_TEST=1 tools/bench_evidence.sh $E/test k_pair_split weak_4096_eps8_test 33554432 $C -- --test-mode || exit 1
NLH_N=8192 NLH_EPS=300 NLH_STEPS=2 tools/bench_evidence.sh $E/eps300 k_prefix_rtw weak_8192_eps300_prod 67108864 $C -- --eps 300 --lattice 8192 --steps 10 --warmup 2 --warmup-ms 0 --no-cpu-baseline || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --test-mode > $E/bench20_test.json 2> $E/bench20_test.err || exit 1
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --strong --lattice 32768 --blocks 2x4 --steps 20 --pmc off --no-cpu-baseline > $E/c3_v8.json 2> $E/c3_v8.err || exit 1
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --map tests/golden/reference_inputs/load_balance_25s_8n.txt --tile 9216 --steps 20 --pmc off --no-cpu-baseline > $E/c5_map.json 2> $E/c5_map.err || exit 1
echo done > $E/done
