set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 240 ./build/pair_bench 4096 200 > $O/pair_bench.jsonl 2> $O/pair_bench.err
