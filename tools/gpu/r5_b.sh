#!/bin/bash
# Round 5, call B: k_pair_split within-block window prefetch (OPT 32) A/B in
# the harness (build/exp/pair_bench_PF = tools/pair_bench.hip -DPB_SET_PF)
set -o pipefail
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 200 build/exp/pair_bench_PF 4096 400 > $O/pf.jsonl 2> $O/pf.err || exit 1
echo done > $O/done
