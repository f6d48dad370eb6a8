set -o pipefail
# round 3: row-pair k_pair_split in libnlh (pair-rows harness at four DMA /
# barrier depths vs the round-3 kernel), the row-pair k_wide harness at C4,
# the GPU suite and the C2 / test-mode benches.  Stops after any step that
# ends in a fault, abort or time limit (exit status other than 0 / 1).
export TMPDIR=/tmp
O=gpurun_out/r3v
mkdir -p $O
timeout -k 10 200 ./build/pair_bench 4096 200 > $O/pair_rows.jsonl 2> $O/pair_rows.err
rc=$?; echo "pair_bench rc=$rc" >> $O/pair_rows.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 ./build/wide_bench 8192 20 > $O/wide_rp.jsonl 2> $O/wide_rp.err
rc=$?; echo "wide_bench rc=$rc" >> $O/wide_rp.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && \
timeout -k 10 400 python bench.py --gpus 1 --steps 1000 --warmup 50 --pmc off --no-cpu-baseline > $O/bench1000.json 2> $O/bench1000.err && \
timeout -k 10 400 python bench.py --gpus 1 --steps 1000 --test-mode --pmc off --no-cpu-baseline > $O/bench_test.json 2> $O/bench_test.err
rc=$?; echo "done rc=$rc" >> $O/smoke.log; exit $rc
