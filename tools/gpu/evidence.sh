#!/bin/bash
# Evidence at a library build (rounds 4-6; replaces the per-call r4_*.sh /
# r5_*.sh scripts, which live in git history):
#   part 1: the whole GPU suite with the per-node / L2 parity records, smoke,
#           the driver's 20-step C2 line three times                 -> SUITE/
#   part 2: per workload a bench line, the rocprofv3 --kernel-trace --stats
#           summary of the same command, PMC passes and record
#           (tools/bench_evidence.sh) for C2, C2 test mode, C4, eps 96,
#           eps 300; C3 on one block and as 8 virtual ranks; the weak
#           layouts as 2 / 4 / 8 virtual ranks                       -> EVID/
#   bash tools/gpu/evidence.sh COMMIT [PART] [SUITE] [EVID]
#   (PART 1 or 2, default both; extra bench.py flags for every line: BENCH_ARGS)
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
PART=${2:-all}
O=${3:-gpurun_out/suite}
E=${4:-gpurun_out/evidence}
B=${BENCH_ARGS:-}
mkdir -p $O $E
if [ "$PART" != 2 ]; then
rm -f gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 $B > $O/bench20_$i.json 2> $O/bench20_$i.err || exit 1
done
echo done > $O/done1
fi
[ "$PART" = 1 ] && exit 0
NLH_N=4096 NLH_EPS=8 tools/bench_evidence.sh $E/c2 k_pair_split weak_4096_eps8_prod 33554432 $C -- $B || exit 1
NLH_N=4096 NLH_EPS=8 NLH_TEST=1 tools/bench_evidence.sh $E/test k_pair_split weak_4096_eps8_test 33554432 $C -- --test-mode $B || exit 1
NLH_N=8192 NLH_EPS=32 tools/bench_evidence.sh $E/c4 k_wide weak_8192_eps32_prod 67108864 $C -- --eps 32 --lattice 8192 --steps 200 $B || exit 1
NLH_N=8192 NLH_EPS=96 NLH_STEPS=6 tools/bench_evidence.sh $E/eps96 k_prefix_rt weak_8192_eps96_prod 67108864 $C -- --eps 96 --lattice 8192 --steps 20 $B || exit 1
NLH_N=8192 NLH_EPS=300 NLH_STEPS=2 tools/bench_evidence.sh $E/eps300 k_prefix_rt weak_8192_eps300_prod 67108864 $C -- --eps 300 --lattice 8192 --steps 4 --warmup 2 --warmup-ms 0 --no-cpu-baseline $B || exit 1
timeout -k 10 300 python bench.py --strong --lattice 32768 --steps 20 --pmc off --no-cpu-baseline $B > $E/c3_1block.json 2> $E/c3_1block.err || exit 1
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --strong --lattice 32768 --blocks 2x4 --steps 20 --pmc off --no-cpu-baseline $B > $E/c3_v8.json 2> $E/c3_v8.err || exit 1
for b in 2x1 2x2 2x4; do
  v=$(( ${b%x*} * ${b#*x} ))
  NLH_VIRTUAL_RANKS=$v timeout -k 10 300 python bench.py --blocks $b --steps 200 --pmc off --no-cpu-baseline $B > $E/weak_v${v}.json 2> $E/weak_v${v}.err || exit 1
done
echo done > $E/done
