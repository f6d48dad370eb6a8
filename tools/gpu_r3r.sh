set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?" >> $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && \
timeout -k 10 1100 bash tools/evidence_r03.sh $O/ev 5f34bc9 > $O/evidence.log 2>&1; echo "evidence rc=$?" >> $O/evidence.log
