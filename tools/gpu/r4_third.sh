#!/bin/bash
# Round 4, third GPU call: the GPU suite after the L2-criterion / balance-test
# fixes (all tests, parity L2 records), k_prefix_rt columns-per-lane harness
# variants, k_wide at eps 40 / 64 after the default-policy DMA change.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 build/prefix_bench 8192 6 48 64 80 96 128 160 > $O/prefix_bench_cpl.jsonl 2> $O/prefix_bench_cpl.err || exit 1
for e in 40 64; do
  timeout -k 10 200 python bench.py --eps $e --lattice 8192 --steps 40 --pmc off --no-cpu-baseline > $O/eps${e}_wide.json 2> $O/eps${e}_wide.err || exit 1
done
echo done > $O/done
