set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3t
mkdir -p $O
timeout -k 10 200 ./build/pair_bench 4096 200 > $O/lag.jsonl 2> $O/lag.err
