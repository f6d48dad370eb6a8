set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
timeout -k 10 200 ./build/pair_bench 4096 200 > $O/mem_abl.jsonl 2> $O/mem_abl.err
