#!/bin/bash
# Round 5, call H: head / interleave / tail options of k_pair_split, ten
# interleaved repetitions (build/exp/pair_bench_TAIL, PB_REPS=10)
set -o pipefail
O=gpurun_out/r5h
mkdir -p $O
PB_REPS=10 timeout -k 10 300 build/exp/pair_bench_TAIL 4096 400 > $O/tail_reps.jsonl 2> $O/tail_reps.err || exit 1
echo done > $O/done
