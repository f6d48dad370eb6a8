#!/bin/bash
# Round 5, call G: OPT 15 / 63 / 79 / 95 interleaved ten times over
# (build/exp/pair_bench_PI, PB_REPS=10), median per variant
set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
PB_REPS=10 timeout -k 10 300 build/exp/pair_bench_PI 4096 400 > $O/pi_reps.jsonl 2> $O/pi_reps.err || exit 1
echo done > $O/done
