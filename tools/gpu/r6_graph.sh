#!/bin/bash
# Round 6: HIP graphs of production passes (NLH_GRAPH) and the new parity
# tests.  1. GPU tests of this round's changes; 2. tools/host_gap.py on C2
# with / without graphs (interleaved, two rounds); 3. per-pass host enqueue
# of C3's 2x4 layout and of 2x2 blocks of 4096^2 as virtual ranks, with /
# without graphs; 4. the driver-form bench line with / without graphs.
#   bash tools/gpu/r6_graph.sh OUTDIR [TESTS]
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6graph}
TESTS=${2:-tests/test_gpu_graph.py tests/test_gpu_stable_dt.py}
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl
timeout -k 10 900 python -u -m pytest $TESTS --maxfail=20 -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log
cp gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl $O/ 2>/dev/null
[ $rc -eq 0 ] || [ "${CONT:-0}" = 1 ] || exit $rc
for round in 1 2; do
  for g in 0 1; do
    NLH_GRAPH=$g timeout -k 10 120 python tools/host_gap.py --reps 60 --label c2_graph$g > $O/c2_graph${g}_$round.jsonl 2> $O/c2_graph${g}_$round.err || exit 1
    tail -1 $O/c2_graph${g}_$round.jsonl
  done
done
for g in 0 1; do
  NLH_GRAPH=$g NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python tools/host_gap.py --reps 8 --lattice 32768 --blocks 2x4 --label c3v8_graph$g > $O/c3v8_graph$g.jsonl 2> $O/c3v8_graph$g.err || exit 1
  tail -1 $O/c3v8_graph$g.jsonl
  NLH_GRAPH=$g NLH_VIRTUAL_RANKS=4 timeout -k 10 200 python tools/host_gap.py --reps 30 --lattice 8192 --blocks 2x2 --label w4_graph$g > $O/w4_graph$g.jsonl 2> $O/w4_graph$g.err || exit 1
  tail -1 $O/w4_graph$g.jsonl
done
for g in 0 1; do
  NLH_GRAPH=$g timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --pmc off --no-cpu-baseline > $O/bench20_graph$g.json 2> $O/bench20_graph$g.err || exit 1
done
echo done > $O/done
