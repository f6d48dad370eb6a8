#!/bin/bash
# rocprofv3 PMC passes over a command, one counter group per pass
# (MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass; at most
# 8 SQ / 4 TCC / 2 GRBM counters per pass).  Each pass under its own timeout.
# Usage: tools/pmc.sh OUTDIR [command ...]   (default command: tools/prof_step.py)
set -u
OUT=${1:-gpurun_out/pmc}
shift || true
if [ $# -eq 0 ]; then set -- python3 tools/prof_step.py; fi
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
  "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
  "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- "$@" > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed: $grp"; exit 1; }
done
echo done
