#!/bin/bash
# Round evidence on one GPU for one workload: the bench.py JSON line, the
# rocprofv3 --kernel-trace --stats summary of the same command, PMC passes
# (tools/pmc.sh) over tools/prof_step.py running the same workload, and the
# PMC record bench.py reads as roofline.physical.
# Usage: tools/bench_evidence.sh OUTDIR KERNEL WKEY NODE_UPDATES_PER_LAUNCH COMMIT -- BENCH_ARGS...
#   prof_step.py takes the workload from NLH_N / NLH_EPS / NLH_TEST / NLH_KERNEL
set -u
O=$1; KERNEL=$2; WKEY=$3; NU=$4; COMMIT=$5; shift 5; [ "${1:-}" = "--" ] && shift
mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 300 python bench.py "$@" > "$O/bench.json" 2> "$O/bench.err" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > "$O/bench_prof.json" 2> "$O/bench_prof.err" || exit 1
tools/pmc.sh "$O/pmc" python3 tools/prof_step.py > "$O/pmc.log" 2>&1 || exit 1
# the per-launch trace is large; the --stats summary is the committed record
rm -f "$O"/prof/*kernel_trace.csv
BID=$(python3 -c "import sys; sys.path.insert(0, '.'); import nonlocalheatequation_amd as N; print(N.build_id())")
python3 tools/pmc_summary.py "$O/pmc" "$KERNEL" --workload "$WKEY" --node-updates "$NU" --commit "$COMMIT" --build-id "$BID" > "$O/pmc_record.json" || exit 1
echo "done $WKEY"
