set -u
O=gpurun_out/v7
mkdir -p $O
timeout -k 10 600 python tools/tune_fast.py --segs 76,102,152 --pair 1 --pair-ablate 12408,10106,10206,10406,10210 --steps 200 > $O/tune_e8.json 2>&1 || exit 1
echo done
