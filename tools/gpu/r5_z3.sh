#!/bin/bash
# Round 5, the build the round ends on (separable test-mode L_h[W0] off
# again): r5_final.sh part 1 (GPU suite, smoke, three 20-step C2 lines), then
# the C2 and test-mode evidence sets (bench line, rocprofv3 stats, PMC)
#   bash tools/gpu/r5_z3.sh COMMIT -> gpurun_out/r5z/, gpurun_out/r5v/{c2,test}
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
E=gpurun_out/r5v
bash tools/gpu/r5_final.sh $C 1 || exit $?
NLH_N=4096 NLH_EPS=8 NLH_TEST=1 tools/bench_evidence.sh $E/test k_pair_split weak_4096_eps8_test 33554432 $C -- --test-mode || exit 1
NLH_N=4096 NLH_EPS=8 tools/bench_evidence.sh $E/c2 k_pair_split weak_4096_eps8_prod 33554432 $C -- || exit 1
echo done > $E/done3
