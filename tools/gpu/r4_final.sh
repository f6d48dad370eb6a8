#!/bin/bash
# Round 4, final GPU call at the library build the round ends on: the whole
# GPU suite (parity L2 records) and smoke, then tools/gpu/r4_evidence.sh
# (bench lines, rocprofv3 stats and PMC records per workload).
#   bash tools/gpu/r4_final.sh COMMIT  -> gpurun_out/r4z/ and gpurun_out/r4e/
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
O=gpurun_out/r4z
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
bash tools/gpu/r4_evidence.sh $C || exit 1
echo done > $O/done
