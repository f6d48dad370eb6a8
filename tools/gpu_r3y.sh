set -o pipefail
# round 3: eps 13 on k_pair_split (row pairs removed its spills) and row pairs
# on k_wide's nested windows past eps 40: GPU suite, smoke, C2 bench line,
# eps 12 / 13 / 14 at 4096^2 and eps 48 / 64 at 8192^2.  Stops after any step
# that ends in a fault, abort or time limit.
export TMPDIR=/tmp
O=gpurun_out/r3y
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && \
for e in 12 13 14; do
  timeout -k 10 300 python bench.py --eps $e --steps 400 --pmc off --no-cpu-baseline > $O/bench_eps$e.json 2> $O/bench_eps$e.err || exit $?
done && \
for e in 48 64; do
  timeout -k 10 300 python bench.py --eps $e --lattice 8192 --steps 20 --pmc off --no-cpu-baseline > $O/bench_eps$e.json 2> $O/bench_eps$e.err || exit $?
done
rc=$?; echo "done rc=$rc" >> $O/smoke.log; exit $rc
