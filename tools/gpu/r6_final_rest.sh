#!/bin/bash
# Round 6, the build the round ends on: the rest of evidence.sh part 2 (C4,
# eps 96, C3 on one block, the weak layouts as 2 / 4 / 8 virtual ranks) and
# the per-horizon prefix lines at eps 1500 / 4000 with rocprofv3 stats.
#   bash tools/gpu/r6_final_rest.sh COMMIT OUT
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
E=${2:-gpurun_out/r6rest}
mkdir -p $E
NLH_N=8192 NLH_EPS=32 tools/bench_evidence.sh $E/c4 k_wide weak_8192_eps32_prod 67108864 $C -- --eps 32 --lattice 8192 --steps 200 || exit 1
NLH_N=8192 NLH_EPS=96 NLH_STEPS=6 tools/bench_evidence.sh $E/eps96 k_prefix_rt weak_8192_eps96_prod 67108864 $C -- --eps 96 --lattice 8192 --steps 20 || exit 1
timeout -k 10 300 python bench.py --strong --lattice 32768 --steps 20 --pmc off --no-cpu-baseline > $E/c3_1block.json 2> $E/c3_1block.err || exit 1
for b in 2x1 2x2 2x4; do
  v=$(( ${b%x*} * ${b#*x} ))
  NLH_VIRTUAL_RANKS=$v timeout -k 10 300 python bench.py --blocks $b --steps 200 --pmc off --no-cpu-baseline > $E/weak_v${v}.json 2> $E/weak_v${v}.err || exit 1
done
for spec in "1500 4096 4" "4000 2048 2"; do
  read -r e n k <<< "$spec"
  mkdir -p $E/eps$e
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/eps$e/prof -o run --output-format csv -- python3 bench.py --eps $e --lattice $n --steps $k --warmup 1 --warmup-ms 0 --pmc off --no-cpu-baseline > $E/eps$e/bench_prof.json 2> $E/eps$e/bench_prof.err || exit 1
  rm -f $E/eps$e/prof/*kernel_trace.csv
done
echo done > $E/done
