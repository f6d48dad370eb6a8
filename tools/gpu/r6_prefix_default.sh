#!/bin/bash
# Round 6: the prefix kernels at the library's default W / R: their GPU tests
# (every form forced too), then one bench line per horizon.
#   bash tools/gpu/r6_prefix_default.sh OUT
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6pdef}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_stable_dt.py tests/test_gpu_parity.py -k "prefix or huge or rtc or knob or unsupported" > $O/pytest.log 2>&1 || exit 1
tail -1 $O/pytest.log
for spec in "96 8192 20" "160 8192 10" "200 8192 10" "300 8192 4" "600 4096 4" "1500 4096 2" "2500 2048 2" "4000 2048 2" "4832 2048 2"; do
  read -r e n k <<< "$spec"
  timeout -k 10 300 python bench.py --eps $e --lattice $n --steps $k --warmup 1 --warmup-ms 0 --pmc off --no-cpu-baseline > $O/e${e}.json 2> $O/e${e}.err || exit 1
  python3 -c "import json; d=json.load(open('$O/e${e}.json')); print($e, round(d['value'],4), round(d['ms_per_step'],3))"
done
echo done > $O/done
