#!/bin/bash
# Round 5, call C: k_pair_split at 1/2/4/6/8 workgroups per CU (segment
# height sized for that many resident workgroups), and the per-wave trace of
# OPT 15 / 7 / 63 / OPT 15 at 8 per CU (build/exp/pair_bench_{OCC,TRACE})
set -o pipefail
O=gpurun_out/r5c
mkdir -p $O
timeout -k 10 200 build/exp/pair_bench_OCC 4096 400 > $O/occ.jsonl 2> $O/occ.err || exit 1
PB_TRACE_DIR=$O timeout -k 10 120 build/exp/pair_bench_TRACE 4096 200 > $O/trace.jsonl 2> $O/trace.err || exit 1
echo done > $O/done
