#!/bin/bash
# Round 5, call R: repartition cost (tools/repart_probe.py, phase trace)
set -o pipefail
O=gpurun_out/r5r
mkdir -p $O
for t in 1024 2048; do
  NLH_VIRTUAL_RANKS=4 NLH_TRACE_REPART=1 timeout -k 10 200 python tools/repart_probe.py $t 3 > $O/probe_$t.jsonl 2> $O/probe_$t.err || exit 1
done
echo done > $O/done
