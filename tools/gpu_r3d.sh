set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?" >> $O/pytest.log
