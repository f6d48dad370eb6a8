set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r3a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a/pytest.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3a/smoke.log 2>&1 && \
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3a/bench20.json 2> gpurun_out/r3a/bench20.err && \
timeout -k 10 200 python bench.py --gpus 1 --steps 1000 --warmup 20 --no-cpu-baseline > gpurun_out/r3a/bench1000.json 2> gpurun_out/r3a/bench1000.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3a/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r3a/bench_prof.json 2> gpurun_out/r3a/bench_prof.err
