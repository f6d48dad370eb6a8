set -u
O=gpurun_out/v3b
mkdir -p $O
timeout -k 10 600 python tools/tune_fast.py --segs 76,100,104,120,137,152,160,180,205 --pair 1 --pair-ablate 1207,1003,1004,1005,1006 --steps 200 > $O/tune_e8.json 2>&1 || exit 1
echo done
