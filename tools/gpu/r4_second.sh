#!/bin/bash
# Round 4, second GPU call (k_wide default-policy DMA, k_prefix_rt NV 6,
# busy test on 8192^2 tiles):
#   1. the whole GPU suite, not stopping at the first failure (parity L2 records)
#   2. smoke, the driver's 20-step C2 line, C4 (8192^2, eps 32)
#   3. the driver's weak-scaling layouts as 2 / 4 / 8 virtual ranks on one GPU
#      (4096^2 per rank, 2x1 / 2x2 / 2x4 blocks): bench lines with the exchange
#      report; the 8-rank one also under rocprofv3 --kernel-trace
#   4. k_prefix_rt at eps 97 .. 224 (NV 6 / 8)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl $O/ 2>/dev/null
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit 1
timeout -k 10 300 python bench.py --eps 32 --lattice 8192 --steps 200 > $O/c4.json 2> $O/c4.err || exit 1
for b in 2x1 2x2 2x4; do
  v=$(( ${b%x*} * ${b#*x} ))
  NLH_VIRTUAL_RANKS=$v timeout -k 10 300 python bench.py --blocks $b --steps 200 --pmc off --no-cpu-baseline > $O/weak_v${v}.json 2> $O/weak_v${v}.err || exit 1
done
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/weak_v8_prof -o run --output-format csv -- python3 bench.py --blocks 2x4 --steps 200 --pmc off --no-cpu-baseline --phase-passes 0 > $O/weak_v8_prof.json 2> $O/weak_v8_prof.err || exit 1
timeout -k 10 300 build/prefix_bench 8192 6 97 128 160 161 192 224 > $O/prefix_bench.jsonl 2> $O/prefix_bench.err || exit 1
for e in 97 128 160 200; do
  timeout -k 10 200 python bench.py --eps $e --lattice 8192 --steps 10 --pmc off --no-cpu-baseline > $O/eps${e}_prefix.json 2> $O/eps${e}_prefix.err || exit 1
done
echo done > $O/done
