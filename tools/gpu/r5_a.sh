#!/bin/bash
# Round 5, call A: the k_pair_split per-wave placement / timing trace at C2,
# and the head-tap skip (OPT 16) A/B in the harness.  (The standalone RCCL
# check ran first in the same script: profiles/r05/rccl/.)  Binaries built on
# the CPU side:
#   build/exp/rccl_p2p_check   (tools/rccl_p2p_check.hip)
#   build/exp/pair_bench_TRACE (tools/pair_bench.hip -DPB_SET_TRACE)
#   build/exp/pair_bench_HEAD  (tools/pair_bench.hip -DPB_SET_HEAD)
set -o pipefail
O=gpurun_out/r5a
mkdir -p $O
PB_TRACE_DIR=$O timeout -k 10 120 build/exp/pair_bench_TRACE 4096 200 > $O/trace.jsonl 2> $O/trace.err || exit 1
timeout -k 10 200 build/exp/pair_bench_HEAD 4096 400 > $O/head.jsonl 2> $O/head.err || exit 1
echo done > $O/done
