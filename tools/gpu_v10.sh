set -u
O=gpurun_out/v10
mkdir -p $O
timeout -k 10 300 python tools/tune_fast.py --segs 0 --pair 1 --steps 200 > $O/tune_normal.json 2>&1 || exit 1
for bs in 0 19 40 76; do
NLH_BAND_SEG=$bs NLH_FORCE_BANDS=1 timeout -k 10 300 python tools/tune_fast.py --segs 0 --pair 1 --steps 200 > $O/tune_bands_$bs.json 2>&1 || exit 1
done
echo done
