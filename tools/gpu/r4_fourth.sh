#!/bin/bash
# Round 4, fourth GPU call: where the virtual-rank busy-timing run diverges
# from one block (tools/diag_busy.py at 2048^2 and 8192^2 tiles), then the
# tests that failed in the third call under the Cauchy-Schwarz L2 regime.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl
timeout -k 10 300 python -u tools/diag_busy.py 2048 > $O/diag_2048.log 2>&1 || exit 1
timeout -k 10 500 python -u tools/diag_busy.py 8192 > $O/diag_8192.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "prefix_rt or weighted" --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl $O/ 2>/dev/null
echo done > $O/done
exit $rc
