#!/bin/bash
# Round 5, call O: the multi-round regime, 343 (no period-aligned rings) with
# the tail skip, lattice-edge select and priority added (build/exp/pair_bench_BIG2)
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
PB_REPS=2 timeout -k 10 400 build/exp/pair_bench_BIG2 16384 100 > $O/big2_16k.jsonl 2> $O/big2_16k.err || exit 1
PB_REPS=2 timeout -k 10 400 build/exp/pair_bench_BIG2 32768 40 > $O/big2_32k.jsonl 2> $O/big2_32k.err || exit 1
echo done > $O/done
