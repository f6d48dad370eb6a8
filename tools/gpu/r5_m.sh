#!/bin/bash
# Round 5, call M: k_prefix_rt partial-horizon rows peeled (PEEL) against the
# round-4 form at eps 65 / 80 / 96 (NV 4), 130 (NV 6), 200 (NV 8), 8192^2
# (build/exp/prefix_bench_PEEL = tools/prefix_bench.hip -DPX_SET_PEEL)
set -o pipefail
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 400 build/exp/prefix_bench_PEEL 8192 10 65 80 96 130 200 > $O/peel.jsonl 2> $O/peel.err || exit 1
echo done > $O/done
