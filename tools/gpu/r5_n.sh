#!/bin/bash
# Round 5, call N: the multi-round regime (one block of 16384^2 / 32768^2,
# launched without the wave priority by the host): round-4 NP against the
# round-5 options (build/exp/pair_bench_BIG)
set -o pipefail
O=gpurun_out/r5n
mkdir -p $O
PB_REPS=2 timeout -k 10 400 build/exp/pair_bench_BIG 16384 100 > $O/big16k.jsonl 2> $O/big16k.err || exit 1
timeout -k 10 400 build/exp/pair_bench_BIG 32768 40 > $O/big32k.jsonl 2> $O/big32k.err || exit 1
echo done > $O/done
