#!/bin/bash
# Round 5, call S: repartitions with the streams, events and staging buffer
# carried over -- the balance tests, the repartition probe, the driver's
# balancing runs of call Q
set -o pipefail
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_balance.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_balance.log 2>&1 || exit 1
for t in 1024 2048; do
  NLH_VIRTUAL_RANKS=4 NLH_TRACE_REPART=1 timeout -k 10 200 python tools/repart_probe.py $t 3 > $O/probe_$t.jsonl 2> $O/probe_$t.err || exit 1
done
bash tools/gpu/r5_q.sh || exit 1
echo done > $O/done
