#!/bin/bash
# Round 4, eighth GPU call: k_pair_split code-shape options in the library
# (incremental store row pointer, unclamped row DMA into padding rows): the
# whole GPU suite, smoke, the driver's 20-step C2 line, C2 over 1000 steps,
# C2 test mode, and the harness again.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc off --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || exit 1
timeout -k 10 300 python bench.py --pmc off --no-cpu-baseline > $O/bench1000.json 2> $O/bench1000.err || exit 1
timeout -k 10 300 python bench.py --test-mode --pmc off --no-cpu-baseline > $O/bench_test.json 2> $O/bench_test.err || exit 1
timeout -k 10 200 build/pair_bench 4096 400 > $O/pair_opt.jsonl 2> $O/pair_opt.err || exit 1
echo done > $O/done
exit $rc
