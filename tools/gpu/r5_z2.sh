#!/bin/bash
# Round 5, last build: the per-workload evidence of r5_final.sh part 2, then
# the kernel-argument placement A/B of r5_kernarg.sh, in one call
#   bash tools/gpu/r5_z2.sh COMMIT
set -o pipefail
bash tools/gpu/r5_final.sh ${1:-unknown} 2 || exit $?
bash tools/gpu/r5_kernarg.sh
