#!/bin/bash
# Round 5, call U: C5 on one GPU -- the reference's uneven map load_balance_25s_8n
# (5x5 tiles of 9216^2 over 8 virtual owners) and the uniform 16384^2-per-owner
# layouts (1x1, 2x4 virtual ranks)
set -o pipefail
O=gpurun_out/r5u
mkdir -p $O
M=tests/golden/reference_inputs/load_balance_25s_8n.txt
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --map $M --tile 9216 --steps 20 --warmup 5 --pmc off --no-cpu-baseline > $O/c5_uneven.json 2> $O/c5_uneven.err || exit 1
timeout -k 10 300 python bench.py --lattice 16384 --steps 20 --warmup 5 --pmc off --no-cpu-baseline > $O/c5_1x1.json 2> $O/c5_1x1.err || exit 1
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --lattice 16384 --blocks 2x4 --steps 20 --warmup 5 --pmc off --no-cpu-baseline > $O/c5_v8.json 2> $O/c5_v8.err || exit 1
echo done > $O/done
