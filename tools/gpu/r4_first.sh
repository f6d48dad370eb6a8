#!/bin/bash
# Round 4, first GPU call after the timing / RCCL-view changes (ABI 9).
#   1. the whole GPU suite (parity L2 records -> parity_l2.jsonl)
#   2. smoke, the driver's 20-step C2 line
#   3. C3 as 8 virtual ranks on one GPU (2x4 blocks of 16384x8192): bench line
#      with the per-pass exchange report, and its rocprofv3 kernel trace
#   4. eps 13 test mode: k_pair_split vs k_fast (NLH_PAIR=0); eps > 64: k_exact vs k_prefix_rt
# Every GPU step under its own time limit; stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --strong --lattice 32768 --blocks 2x4 --steps 40 --pmc off --no-cpu-baseline > $O/c3_v8.json 2> $O/c3_v8.err || exit 1
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3_v8_prof -o run --output-format csv -- python3 bench.py --strong --lattice 32768 --blocks 2x4 --steps 40 --pmc off --no-cpu-baseline --phase-passes 0 > $O/c3_v8_prof.json 2> $O/c3_v8_prof.err || exit 1
timeout -k 10 200 python bench.py --strong --lattice 32768 --steps 40 --pmc off --no-cpu-baseline > $O/c3_1block.json 2> $O/c3_1block.err || exit 1
timeout -k 10 200 python bench.py --eps 13 --test-mode --steps 400 --pmc off --no-cpu-baseline > $O/eps13_test_pair.json 2> $O/eps13_test_pair.err || exit 1
NLH_PAIR=0 timeout -k 10 200 python bench.py --eps 13 --test-mode --steps 400 --pmc off --no-cpu-baseline > $O/eps13_test_fast.json 2> $O/eps13_test_fast.err || exit 1
timeout -k 10 300 python bench.py --eps 80 --lattice 8192 --steps 4 --warmup 1 --warmup-ms 0 --pmc off --no-cpu-baseline --kernel exact > $O/eps80_exact.json 2> $O/eps80_exact.err || exit 1
timeout -k 10 300 python bench.py --eps 96 --lattice 8192 --steps 2 --warmup 1 --warmup-ms 0 --pmc off --no-cpu-baseline --kernel exact > $O/eps96_exact.json 2> $O/eps96_exact.err || exit 1
for e in 65 80 96 97 128; do
  timeout -k 10 200 python bench.py --eps $e --lattice 8192 --steps 20 --pmc off --no-cpu-baseline > $O/eps${e}_prefix.json 2> $O/eps${e}_prefix.err || exit 1
done
timeout -k 10 300 build/wide_bench_wpg 8192 20 > $O/wide_wpg.jsonl 2> $O/wide_wpg.err || exit 1
timeout -k 10 300 build/prefix_bench 8192 10 32 40 48 56 64 80 96 128 > $O/prefix_bench.jsonl 2> $O/prefix_bench.err || exit 1
echo done > $O/done
