#!/bin/bash
# Round 5, call L: period-aligned rings (OPT 2048) A/B (build/exp/pair_bench_RING, PB_REPS=8)
set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
PB_REPS=8 timeout -k 10 300 build/exp/pair_bench_RING 4096 400 > $O/ring_reps2.jsonl 2> $O/ring_reps2.err || exit 1
echo done > $O/done
