set -u
O=gpurun_out/v8
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiblock.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
NLH_PAIR_SPLIT=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiblock.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_mw.log 2>&1 || { echo pytest mw failed; tail -30 $O/pytest_mw.log; exit 1; }
tail -1 $O/pytest.log; tail -1 $O/pytest_mw.log
timeout -k 10 300 python tools/tune_fast.py --segs 76,137,152 --pair 1 --steps 200 > $O/tune_split.json 2>&1 || exit 1
NLH_PAIR_SPLIT=2 timeout -k 10 300 python tools/tune_fast.py --segs 76,102,137,152,160 --pair 1 --steps 200 > $O/tune_mw.json 2>&1 || exit 1
echo done
