#!/bin/bash
# Round 5, call D: k_pair_split row pairs' levels interleaved (OPT 64) A/B
# (build/exp/pair_bench_PI = tools/pair_bench.hip -DPB_SET_PI)
set -o pipefail
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 200 build/exp/pair_bench_PI 4096 400 > $O/pi.jsonl 2> $O/pi.err || exit 1
echo done > $O/done
