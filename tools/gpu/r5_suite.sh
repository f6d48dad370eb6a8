#!/bin/bash
# Round 5: the whole GPU suite (full-length C2 / C3 parity, per-node relative
# error records), smoke, the driver's 20-step C2 line twice, and the C2
# evidence set (bench line, rocprofv3 --kernel-trace --stats, PMC record).
#   bash tools/gpu/r5_suite.sh COMMIT -> gpurun_out/r5s/, gpurun_out/r5s/c2/
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
O=gpurun_out/r5s
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --pmc off > $O/bench20_b.json 2> $O/bench20_b.err || exit 1
NLH_N=4096 NLH_EPS=8 tools/bench_evidence.sh $O/c2 k_pair_split weak_4096_eps8_prod 33554432 $C -- || exit 1
echo done > $O/done
