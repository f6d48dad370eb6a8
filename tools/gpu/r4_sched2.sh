#!/bin/bash
# Round 4: NLH_INT_PER_CU / NLH_COMM_PRIO on per-rank-sized (4096^2) blocks:
# 8192x4096 as 2x1 and 8192^2 as 2x2 blocks over RCCL to self; repeated.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python -u tools/diag_sched.py 200 2x1 8192x4096 short >> $O/sched_4096blocks.jsonl 2>> $O/sched.err || exit 1
  timeout -k 10 300 python -u tools/diag_sched.py 100 2x2 8192x8192 short >> $O/sched_4096blocks.jsonl 2>> $O/sched.err || exit 1
  timeout -k 10 300 python -u tools/diag_sched.py 200 2x1 4096x4096 short >> $O/sched_2048blocks.jsonl 2>> $O/sched.err || exit 1
done
echo done > $O/done
