set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_balance.py -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?" >> $O/pytest.log
