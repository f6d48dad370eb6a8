#!/bin/bash
# Round 5, call T: k_prefix_rt with two output columns per lane (PX_SET_CPL)
set -o pipefail
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 400 build/exp/prefix_bench_CPL 8192 10 65 80 96 128 160 > $O/cpl.jsonl 2> $O/cpl.err || exit 1
echo done > $O/done
