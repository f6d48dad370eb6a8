#!/bin/bash
# Round 5: the production pass compiled with different AMDGPU scheduling
# strategies (pair_bench -DPB_SET_ONE, one binary per option), interleaved
set -o pipefail
O=gpurun_out/r5s2
mkdir -p $O
for rep in 1 2 3 4; do
  for b in default maxilp itilp memclause bias0; do
    timeout -k 10 120 build/exp/pb_$b 4096 300 >> $O/sched.jsonl 2>> $O/sched.err || exit 1
  done
done
echo done > $O/done
