#!/bin/bash
# Round 5, call K: wave priority and stage-1 lean periods under OPT 223
# (build/exp/pair_bench_W0, PB_REPS=8)
set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
PB_REPS=8 timeout -k 10 300 build/exp/pair_bench_W0 4096 400 > $O/w0_reps.jsonl 2> $O/w0_reps.err || exit 1
echo done > $O/done
