set -o pipefail
# round 3: k_wide row-pair sweeps -- eps 32 (D / PA / CH with row pairs vs
# one row) and the nested-window path at eps 48 / 64 (one row vs row pairs)
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
timeout -k 10 240 ./build/wide_bench_32 8192 20 > $O/wide32.jsonl 2> $O/wide32.err
rc=$?; echo "rc=$rc" >> $O/wide32.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 ./build/wide_bench_48 8192 10 > $O/wide48.jsonl 2> $O/wide48.err
rc=$?; echo "rc=$rc" >> $O/wide48.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 ./build/wide_bench_64 8192 10 > $O/wide64.jsonl 2> $O/wide64.err
rc=$?; echo "rc=$rc" >> $O/wide64.err; exit $rc
