#!/bin/bash
# Round 6: the driver's exact bench command three times on one box (the
# spread of the 20-step line across boxes: run once per call).
#   bash tools/gpu/r6_lines.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6lines}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$i.json 2> $O/bench20_$i.err || exit 1
  python3 -c "import json; d=json.load(open('$O/bench20_$i.json')); print(round(d['value'],1), round(d['roofline']['kernel_avg_us'],2), round(d['host']['outside_events_us'],1))"
done
rocm-smi --showproductname > $O/smi.txt 2>&1 || true
echo done > $O/done
