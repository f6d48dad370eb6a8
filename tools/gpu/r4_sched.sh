#!/bin/bash
# Round 4: exchange-path schedule knobs on a per-rank proxy of the weak bench
# (tools/diag_sched.py), 2x1 and 2x2 blocks over RCCL to self.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 400 python -u tools/diag_sched.py 200 2x1 > $O/sched_2x1.jsonl 2> $O/sched.err || exit 1
timeout -k 10 400 python -u tools/diag_sched.py 200 2x2 > $O/sched_2x2.jsonl 2>> $O/sched.err || exit 1
echo done > $O/done
