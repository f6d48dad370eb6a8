#!/bin/bash
# Round 5, call V: k_prefix_rt table prefetch (TPRE) and batched LDS reads (BATCH)
set -o pipefail
O=gpurun_out/r5v2
mkdir -p $O
timeout -k 10 500 build/exp/prefix_bench_TB 8192 10 65 80 96 128 160 200 > $O/tb.jsonl 2> $O/tb.err || exit 1
echo done > $O/done
