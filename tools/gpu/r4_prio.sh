#!/bin/bash
# Round 4: k_pair_split wave priority (OPT 7 vs 15) and the ring depth /
# barrier block under it, C2 block in the harness.  Build first (CPU):
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPB_SET_PRIO (or -DPB_SET_DB) -Iinclude \
#     -Inonlocalheatequation_amd/csrc -mllvm -pragma-unroll-threshold=1000000 \
#     tools/pair_bench.hip -o build/pair_bench_PRIO (build/pair_bench_DB)
set -o pipefail
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 200 build/pair_bench_PRIO 4096 400 > $O/prio_lib.jsonl 2> $O/prio_lib.err || exit 1
timeout -k 10 200 build/pair_bench_PRIO 4096 400 >> $O/prio_lib.jsonl 2>> $O/prio_lib.err || exit 1
echo done > $O/done
