#!/bin/bash
# Round 4: one C3 rank's 16384 x 8192 block alone on one GPU (pass time), and
# with the exchange-path schedule forced on (bands on all four sides).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 300 python -u tools/diag_sched.py 40 1x1 16384x8192 short > $O/c3rank.jsonl 2> $O/c3rank.err || exit 1
NLH_FORCE_BANDS=1 timeout -k 10 300 python -u tools/diag_sched.py 40 1x1 16384x8192 short > $O/c3rank_bands.jsonl 2>> $O/c3rank.err || exit 1
echo done > $O/done
