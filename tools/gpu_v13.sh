set -u
O=gpurun_out/v13
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiblock.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for n in 4096 8192 16384 32768; do
timeout -k 10 300 python tools/tune_eps.py --n $n --eps 8 --steps 20 --rounds 2 >> $O/sizes_e8.jsonl 2>&1 || exit 1
done
echo done
