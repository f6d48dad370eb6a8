#!/bin/bash
# Round 6 trial (a build with the NLH_EVFENCE knob; adopted for the two
# per-pass events ev_band / ev_int, the knob removed): the exchange schedule's
# stream-order events created with hipEventDisableSystemFence (device-scope
# release / acquire) on the rank proxies and the virtual-rank lines, parity
# tests of the multi-block paths.
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6evf}; mkdir -p $O
NLH_EVFENCE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_configs.py -k "knob or blocks or virtual" > $O/pytest.log 2>&1 || exit 1
tail -1 $O/pytest.log
bash tools/gpu/r6_band_sched.sh $O/lines "one:NLH_X=0" "m4:NLH_FORCE_BANDS=4" "m4f:NLH_FORCE_BANDS=4,NLH_EVFENCE=1" "m26:NLH_FORCE_BANDS=26" "m26f:NLH_FORCE_BANDS=26,NLH_EVFENCE=1" "v8:NLH_VIRTUAL_RANKS=8" "v8f:NLH_VIRTUAL_RANKS=8,NLH_EVFENCE=1" || exit 1
