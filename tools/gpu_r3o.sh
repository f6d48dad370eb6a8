set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 200 ./build/pair_bench 4096 200 > $O/barrier_abl.jsonl 2> $O/barrier_abl.err
