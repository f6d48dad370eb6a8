#!/bin/bash
# Round evidence on one GPU: bench JSON line, rocprofv3 kernel-trace stats of
# the same command, PMC traffic passes + their summary for the dominant
# kernel.  Usage: tools/bench_evidence.sh TAG [KERNEL_MATCH]
set -u
TAG=${1:-r01}
KEY=${2:-k_pair}
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python bench.py --no-cpu-baseline > "$O/bench_prof.json" 2> "$O/bench_prof.err" || exit 1
tools/pmc.sh "$O/pmc" > "$O/pmc.log" 2>&1 || exit 1
python tools/pmc_summary.py "$O/pmc" "$KEY" > "$O/pmc_summary.json" || exit 1
echo done
