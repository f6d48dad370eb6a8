#!/bin/bash
# Round 5, call F: k_pair_split ablations (build/exp/pair_bench_ABL): timing,
# then the PMC passes of r5_e.sh over the same binary
set -o pipefail
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 200 build/exp/pair_bench_ABL 4096 400 > $O/abl.jsonl 2> $O/abl.err || exit 1
O=$O/pmc BIN=build/exp/pair_bench_ABL bash tools/gpu/r5_e.sh || exit 1
echo done > gpurun_out/r5f/done
