set -u
O=gpurun_out/v4
mkdir -p $O
NLH_PAIR_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiblock.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_split.log 2>&1 || { echo pytest failed; tail -30 $O/pytest_split.log; exit 1; }
tail -2 $O/pytest_split.log
NLH_PAIR_SPLIT=1 timeout -k 10 600 python tools/tune_fast.py --segs 76,137,148,152,156,160,168 --pair 1 --pair-ablate 1207,1003,1004,1005,1007 --steps 200 > $O/tune_e8.json 2>&1 || exit 1
NLH_PAIR_SPLIT=1 timeout -k 10 300 python tools/tune_eps.py --eps 1-16 --steps 200 > $O/tune_eps_split.jsonl 2>&1 || exit 1
echo done
