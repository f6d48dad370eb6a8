set -u
O=gpurun_out/v3
mkdir -p $O
NLH_PAIR_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiblock.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_split.log 2>&1 || { echo pytest failed; tail -30 $O/pytest_split.log; exit 1; }
tail -2 $O/pytest_split.log
timeout -k 10 300 python tools/tune_fast.py --segs 76,80,96,112,128,152 --pair 1 --pair-ablate 207,1207,1004 > $O/tune_e8.json 2>&1 || exit 1
NLH_PAIR_SPLIT=1 timeout -k 10 300 python tools/tune_fast.py --segs 38,40,48,64,76,80,96 --pair 1 > $O/tune_e8_split.json 2>&1 || exit 1
NLH_PAIR_SPLIT=1 timeout -k 10 300 python tools/tune_eps.py --eps 1-16 --steps 100 > $O/tune_eps_split.jsonl 2>&1 || exit 1
echo done
