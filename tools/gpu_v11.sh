set -u
O=gpurun_out/v11
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiblock.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/tune_fast.py --segs 0 --pair 1 --steps 200 > $O/tune_normal.json 2>&1 || exit 1
for bs in 0 19 40 76; do
NLH_BAND_SEG=$bs NLH_FORCE_BANDS=1 timeout -k 10 300 python tools/tune_fast.py --segs 0 --pair 1 --steps 200 > $O/tune_bands_$bs.json 2>&1 || exit 1
done
echo done
