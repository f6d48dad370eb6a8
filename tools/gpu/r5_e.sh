#!/bin/bash
# Round 5, call E: PMC passes over the k_pair_split harness variants
# (OPT 15 / 63 / 79 / 95; build/exp/pair_bench_PI), one counter group per
# pass, summarised per kernel symbol by tools/pmc_kernels.py
set -o pipefail
O=${O:-gpurun_out/r5e}
BIN=${BIN:-build/exp/pair_bench_PI}
mkdir -p $O
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
  "SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM" \
  "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $O/p$i -o run -- $BIN 4096 20 > $O/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 tools/pmc_kernels.py $O > $O/summary.json || exit 1
echo done > $O/done
