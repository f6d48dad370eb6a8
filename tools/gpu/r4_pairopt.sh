#!/bin/bash
# Round 4: k_pair_split code-shape options (incremental store row pointer,
# unclamped row DMA into padding rows) in the harness, C2 block, bitwise
# against the unoptimised form.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 200 build/pair_bench 4096 200 > $O/pair_opt.jsonl 2> $O/pair_opt.err || exit 1
timeout -k 10 200 build/pair_bench 4096 200 > $O/pair_opt_2.jsonl 2>> $O/pair_opt.err || exit 1
echo done > $O/done
