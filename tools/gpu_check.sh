#!/bin/bash
# One GPU session: parity + multi-block tests, bandwidth probe, fast-kernel
# tuning sweep at eps=8 and eps=32.  Every GPU step has its own time limit
# and the script stops at the first failure.  Usage: tools/gpu_check.sh TAG
set -u
TAG=${1:-x}
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py tests/test_gpu_multiblock.py -q -x -p no:cacheprovider > "$O/pytest.log" 2>&1
echo "pytest rc=$?" >> "$O/pytest.log"
tail -1 "$O/pytest.log" | grep -q "rc=0" || exit 1
if [ -x build/issue_probe ]; then timeout -k 10 120 build/issue_probe > "$O/issue.txt" 2>&1 || exit 1; fi
if [ -x build/bw_probe ]; then timeout -k 10 300 build/bw_probe > "$O/bw.txt" 2>&1 || exit 1; fi
timeout -k 10 300 python tools/tune_fast.py --segs 64,128,256 > "$O/tune_e8.json" 2>&1 || exit 1
timeout -k 10 300 python tools/tune_fast.py --eps 32 --n 8192 --segs 512,1024,2048 --steps 10 > "$O/tune_e32.json" 2>&1 || exit 1
echo done
