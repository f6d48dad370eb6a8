#!/bin/bash
# Round 5, call J: eight s_nop per row on wave 0 / wave 1 of OPT 223
# (build/exp/pair_bench_NOP, PB_REPS=8)
set -o pipefail
O=gpurun_out/r5j
mkdir -p $O
PB_REPS=8 timeout -k 10 300 build/exp/pair_bench_NOP 4096 400 > $O/nop_reps.jsonl 2> $O/nop_reps.err || exit 1
echo done > $O/done
