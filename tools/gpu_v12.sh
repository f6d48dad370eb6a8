set -u
O=gpurun_out/v12
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_fullsize.log 2>&1 || { echo pytest failed; tail -30 $O/pytest_fullsize.log; exit 1; }
tail -3 $O/pytest_fullsize.log
timeout -k 10 300 python tools/tune_eps.py --n 16384 --eps 8 --steps 20 --rounds 2 > $O/c5_16384.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/tune_eps.py --n 32768 --eps 8 --steps 10 --rounds 2 > $O/c3_32768.jsonl 2>&1 || exit 1
timeout -k 10 300 python tools/tune_eps.py --n 8192 --eps 32 --steps 10 --rounds 2 > $O/c4_8192_e32.jsonl 2>&1 || exit 1
echo done
