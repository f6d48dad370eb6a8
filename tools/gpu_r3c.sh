set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?" >> $O/pytest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --warmup-ms 0 --pmc off --no-cpu-baseline > $O/bench20_nowarm.json 2> $O/bench20_nowarm.err && \
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 --pmc off --no-cpu-baseline > $O/bench1000.json 2> $O/bench1000.err && \
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 10 --eps 32 --lattice 8192 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 4 --eps 56 --lattice 8192 --pmc off --no-cpu-baseline > $O/bench_eps56.json 2> $O/bench_eps56.err && \
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 4 --eps 64 --lattice 8192 --pmc off --no-cpu-baseline > $O/bench_eps64.json 2> $O/bench_eps64.err
