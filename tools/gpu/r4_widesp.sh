#!/bin/bash
# Round 4: k_wide with a per-chunk output row pointer (SP) against the
# per-store row multiply, C4 block in the harness.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 300 build/wide_bench 8192 40 > $O/wide_sp.jsonl 2> $O/wide_sp.err || exit 1
timeout -k 10 300 build/wide_bench 8192 40 > $O/wide_sp_2.jsonl 2>> $O/wide_sp.err || exit 1
echo done > $O/done
