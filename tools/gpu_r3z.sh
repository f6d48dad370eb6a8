set -o pipefail
# round 3, last call: the GPU tests of the kernels the last library change
# touched (k_pair_split at eps 13, k_wide nested windows past eps 40), smoke,
# the C2 bench line and eps 13 / 64.  Stops after any fault, abort or time limit.
export TMPDIR=/tmp
O=gpurun_out/r3z
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc off > $O/bench20.json 2> $O/bench20.err && \
timeout -k 10 200 python bench.py --eps 13 --steps 400 --pmc off --no-cpu-baseline > $O/bench_eps13.json 2> $O/bench_eps13.err && \
timeout -k 10 200 python bench.py --eps 64 --lattice 8192 --steps 20 --pmc off --no-cpu-baseline > $O/bench_eps64.json 2> $O/bench_eps64.err
rc=$?; echo "done rc=$rc" >> $O/smoke.log; exit $rc
