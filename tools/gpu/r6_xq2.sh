#!/bin/bash
# Round 6 trial (a library build with the NLH_XQ knob under the bands-own-
# stream schedule, removed again after this run): memory-value waits vs event
# waits on the 4096^2 rank proxies, with a kernel trace.  Result: worse
# (profiles/r06/rank_proxy/timeline/).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6xq2; mkdir -p $O
NLH_XQ=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "knob or blocks" > $O/pytest.log 2>&1 || exit 1
tail -1 $O/pytest.log
bash tools/gpu/r6_band_sched.sh $O/lines "one:NLH_X=0" "m4:NLH_FORCE_BANDS=4" "m4xq:NLH_FORCE_BANDS=4,NLH_XQ=1" "m26:NLH_FORCE_BANDS=26" "m26xq:NLH_FORCE_BANDS=26,NLH_XQ=1" "v8:NLH_VIRTUAL_RANKS=8" "v8xq:NLH_VIRTUAL_RANKS=8,NLH_XQ=1" || exit 1
NLH_FORCE_BANDS=4 NLH_XQ=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tl -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --warmup-ms 100 --pmc off --no-cpu-baseline --phase-passes 0 > $O/tl.json 2> $O/tl.err || exit 1
