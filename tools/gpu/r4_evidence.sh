#!/bin/bash
# Round 4 evidence at the library build the round ends on: per workload the
# bench line, the rocprofv3 --kernel-trace --stats summary of the same
# command, PMC passes over tools/prof_step.py and the PMC record
# (tools/bench_evidence.sh), and the driver's 20-step C2 line.  The GPU suite
# and smoke at the same build run in their own call (tools/gpu/r4_fifth.sh).
#   bash tools/gpu/r4_evidence.sh COMMIT   -> gpurun_out/r4e/<workload>/
# committed as profiles/r04/evidence/; the PMC records also as profiles/pmc/.
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
O=gpurun_out/r4e
mkdir -p $O
NLH_N=4096 NLH_EPS=8 tools/bench_evidence.sh $O/c2 k_pair_split weak_4096_eps8_prod 33554432 $C -- || exit 1
NLH_N=4096 NLH_EPS=8 NLH_TEST=1 tools/bench_evidence.sh $O/test k_pair_split weak_4096_eps8_test 33554432 $C -- --test-mode || exit 1
NLH_N=8192 NLH_EPS=32 tools/bench_evidence.sh $O/c4 k_wide weak_8192_eps32_prod 67108864 $C -- --eps 32 --lattice 8192 --steps 200 || exit 1
NLH_N=8192 NLH_EPS=40 tools/bench_evidence.sh $O/eps40 k_wide weak_8192_eps40_prod 67108864 $C -- --eps 40 --lattice 8192 --steps 100 || exit 1
NLH_N=8192 NLH_EPS=64 tools/bench_evidence.sh $O/eps64 k_wide weak_8192_eps64_prod 67108864 $C -- --eps 64 --lattice 8192 --steps 40 || exit 1
NLH_N=8192 NLH_EPS=96 NLH_STEPS=6 tools/bench_evidence.sh $O/eps96 k_prefix_rt weak_8192_eps96_prod 67108864 $C -- --eps 96 --lattice 8192 --steps 20 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
echo done > $O/done
