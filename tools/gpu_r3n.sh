set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
for cfg in "4096 200 0" "4096 200 76" "4096 200 304" "8192 100 152" "8192 100 304" "8192 100 608" "8192 100 1216"; do
  timeout -k 10 120 ./build/pair_bench $cfg >> $O/seg_sweep.jsonl 2>> $O/seg_sweep.err || exit 1
done
