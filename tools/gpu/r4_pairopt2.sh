#!/bin/bash
# Round 4: k_pair_split single-column store behind a wave-uniform test
# (OPT 4) on top of the production row pointer (OPT 1), C2 harness.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
timeout -k 10 200 build/pair_bench 4096 400 > $O/pair_opt2.jsonl 2> $O/pair_opt2.err || exit 1
timeout -k 10 200 build/pair_bench 4096 400 > $O/pair_opt2_b.jsonl 2>> $O/pair_opt2.err || exit 1
echo done > $O/done
