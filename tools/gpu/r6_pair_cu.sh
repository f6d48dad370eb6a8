set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6paircu; mkdir -p $O
for rep in 1 2 3; do
for cu in 4 5 3; do
  NLH_PAIR_CU=$cu timeout -k 10 120 python bench.py --steps 200 --warmup 20 --pmc off --no-cpu-baseline > $O/cu${cu}_$rep.json 2> $O/cu${cu}_$rep.err || exit 1
  python3 -c "import json; d=json.load(open('$O/cu${cu}_$rep.json')); print($cu, $rep, round(d['value'],1), round(d['roofline']['kernel_avg_us'],2))"
done
done
