#!/bin/bash
# Round 5, call Z: wave 1's priority raised only around its DMA and window
# reads (pair_bench -DPB_SET_PRIO2), C2 block, variants interleaved 4 times
set -o pipefail
O=gpurun_out/r5zz
mkdir -p $O
PB_REPS=4 timeout -k 10 400 build/exp/pair_bench_PRIO2 4096 300 > $O/prio2.jsonl 2> $O/prio2.err || exit 1
echo done > $O/done
