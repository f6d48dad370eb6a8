set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3q
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -k "large_eps or wide" -v --timeout 200 --timeout-method thread > $O/pytest_wide.log 2>&1; echo "pytest rc=$?" >> $O/pytest_wide.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 4 --eps 56 --lattice 8192 --pmc off --no-cpu-baseline > $O/bench_eps56.json 2> $O/bench_eps56.err && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 4 --eps 64 --lattice 8192 --pmc off --no-cpu-baseline > $O/bench_eps64.json 2> $O/bench_eps64.err && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 4 --eps 49 --lattice 8192 --pmc off --no-cpu-baseline > $O/bench_eps49.json 2> $O/bench_eps49.err
