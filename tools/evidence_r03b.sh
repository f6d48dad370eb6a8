#!/bin/bash
# Round-3 evidence after the row-pair kernels: bench line + rocprofv3 stats +
# PMC for C2 (k_pair_split), C2 test mode and C4 (k_wide eps 32).
# Usage: tools/evidence_r03b.sh OUTROOT COMMIT
set -u
O=$1; C=$2
NLH_N=4096 NLH_EPS=8 tools/bench_evidence.sh "$O/c2" k_pair_split weak_4096_eps8_prod 33554432 "$C" -- || exit 1
NLH_N=4096 NLH_EPS=8 NLH_TEST=1 tools/bench_evidence.sh "$O/test" k_pair_split weak_4096_eps8_test 33554432 "$C" -- --test-mode || exit 1
NLH_N=8192 NLH_EPS=32 tools/bench_evidence.sh "$O/c4" k_wide weak_8192_eps32_prod 67108864 "$C" -- --eps 32 --lattice 8192 --steps 200 || exit 1
echo evidence done
