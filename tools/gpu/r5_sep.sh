#!/bin/bash
# Round 5: the separable L_h[W0] test-mode pass in the library -- GPU suite,
# smoke, the test-mode evidence set, the 20-step C2 line, and the harness A/B
#   bash tools/gpu/r5_sep.sh COMMIT
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
O=gpurun_out/r5sep
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
NLH_N=4096 NLH_EPS=8 NLH_TEST=1 tools/bench_evidence.sh $O/test k_pair_split weak_4096_eps8_test 33554432 $C -- --test-mode || exit 1
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$i.json 2> $O/bench20_$i.err || exit 1
done
echo done > $O/done
