set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 240 ./build/pair_bench 4096 200 > $O/pair_bench.jsonl 2> $O/pair_bench.err && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "pair or fast" -x -q --timeout 120 --timeout-method thread > $O/pytest_pair.log 2>&1; echo "rc=$?" >> $O/pytest_pair.log
