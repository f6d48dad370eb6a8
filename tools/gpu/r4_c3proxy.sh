#!/bin/bash
# Round 4: C3's per-rank block (16384 x 8192) beside an exchange: 16384^2 as
# 1x2 and 32768 x 16384 as 2x2 blocks over RCCL to self (tools/diag_sched.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 400 python -u tools/diag_sched.py 40 1x2 16384x16384 short > $O/c3proxy_1x2.jsonl 2> $O/c3proxy.err || exit 1
timeout -k 10 400 python -u tools/diag_sched.py 20 2x2 32768x16384 short > $O/c3proxy_2x2.jsonl 2>> $O/c3proxy.err || exit 1
echo done > $O/done
