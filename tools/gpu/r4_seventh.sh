#!/bin/bash
# Round 4, seventh GPU call: chunked messages + new blocks zeroed on their own stream (diagnostic at
# 8192^2 tiles, then the balance tests), then the whole GPU suite and smoke.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl
timeout -k 10 500 python -u tools/diag_busy.py 8192 > $O/diag_8192.log 2>&1 || exit 1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; echo "smoke rc=$?" >> $O/smoke.log
echo done > $O/done
exit $rc
