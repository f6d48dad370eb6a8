#!/bin/bash
# Round 4: host enqueue time per pass against GPU time per pass for the
# multi-GPU bench layouts (tools/diag_enqueue.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 300 python -u tools/diag_enqueue.py 20 > $O/enqueue.jsonl 2> $O/enqueue.err || exit 1
timeout -k 10 300 python -u tools/diag_enqueue.py 200 > $O/enqueue_200.jsonl 2>> $O/enqueue.err || exit 1
echo done > $O/done
