set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 300 ./build/wide_bench 8192 20 > $O/wide_bench.jsonl 2> $O/wide_bench.err
