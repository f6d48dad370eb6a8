set -u
O=gpurun_out/v6
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiblock.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python tools/tune_fast.py --segs 76,152,156,160 --pair 1 --pair-ablate 1207,1004,1006,1010,1012 --steps 200 > $O/tune_e8.json 2>&1 || exit 1
timeout -k 10 300 python tools/tune_eps.py --eps 1-16 --steps 200 > $O/tune_eps.jsonl 2>&1 || exit 1
echo done
