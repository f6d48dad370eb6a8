# Round evidence: full GPU test suite, bench line, rocprofv3 stats, PMC.
# Usage: tools/gpu_ev.sh TAG [KERNEL_MATCH]
set -u
TAG=${1:-ev}
KEY=${2:-k_pair_split}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
tools/bench_evidence.sh $TAG/ev $KEY || exit 1
echo done
