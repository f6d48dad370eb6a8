#!/bin/bash
# Round 5: what the test-mode pass's L_h[W0] row DMA costs (pair_bench -DPB_SET_TESTABL)
set -o pipefail
O=gpurun_out/r5ta
mkdir -p $O
PB_REPS=4 timeout -k 10 400 build/exp/pair_bench_TESTABL 4096 300 > $O/testabl.jsonl 2> $O/testabl.err || exit 1
echo done > $O/done
