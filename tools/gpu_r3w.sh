set -o pipefail
# round 3: libnlh with row pairs in k_pair_split (8-slot rings by default) and
# k_wide (production, E <= 32): GPU suite, smoke, the driver's bench line, and
# the evidence (bench + rocprofv3 stats + PMC) for C2, C2 test mode and C4.
# Stops after any step that ends in a fault, abort or time limit.
export TMPDIR=/tmp
O=gpurun_out/r3w
C=${1:-HEAD}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && \
timeout -k 10 400 python bench.py --gpus 1 --steps 1000 --warmup 50 --pmc off --no-cpu-baseline > $O/bench1000.json 2> $O/bench1000.err && \
timeout -k 10 1000 bash tools/evidence_r03b.sh $O/ev $C > $O/evidence.log 2>&1
rc=$?; echo "done rc=$rc" >> $O/smoke.log; exit $rc
