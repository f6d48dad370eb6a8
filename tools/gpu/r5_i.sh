#!/bin/bash
# Round 5, call I: DMA rows in flight under OPT 223 (PB_REPS=8), and the
# per-wave trace of OPT 15 / 31 / 7 / 63 / 223 / 223 at D = 8
set -o pipefail
O=gpurun_out/r5i
mkdir -p $O
PB_REPS=8 timeout -k 10 300 build/exp/pair_bench_DEPTH 4096 400 > $O/depth_reps.jsonl 2> $O/depth_reps.err || exit 1
PB_TRACE_DIR=$O timeout -k 10 120 build/exp/pair_bench_TRACE 4096 200 > $O/trace.jsonl 2> $O/trace.err || exit 1
echo done > $O/done
