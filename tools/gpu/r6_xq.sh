#!/bin/bash
# Round 6 trial (library build with the NLH_XQ knob, removed again after this
# run): the exchange schedule's cross-queue waits as stream memory-value waits
# (hipStreamWaitValue32 / hipStreamWriteValue32 on pass counters in signal
# memory) instead of event waits, on the four-sided and bottom-only rank
# proxies and 2 virtual ranks.  Result: equal (profiles/r06/rank_proxy/xq/).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6xq; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "NLH_XQ or FORCE_BANDS" > $O/pytest.log 2>&1 || exit 1
tail -1 $O/pytest.log
bash tools/gpu/r6_band_sched.sh $O/lines "one:NLH_X=0" "fb:NLH_FORCE_BANDS=1" "fbxq:NLH_FORCE_BANDS=1,NLH_XQ=1" "b:NLH_FORCE_BANDS=16" "bxq:NLH_FORCE_BANDS=16,NLH_XQ=1" "v2:NLH_VIRTUAL_RANKS=2" "v2xq:NLH_VIRTUAL_RANKS=2,NLH_XQ=1" || exit 1
