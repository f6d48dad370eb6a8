set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 200 ./build/wide_bench_56 8192 10 > $O/wide56.jsonl 2> $O/wide56.err && \
timeout -k 10 200 ./build/wide_bench_64 8192 10 > $O/wide64.jsonl 2> $O/wide64.err
