#!/bin/bash
# Round 4, final GPU call after the interior-slot default change: the whole
# GPU suite and smoke, tools/gpu/r4_evidence.sh, and the multi-rank layouts
# on one GPU (weak 2x1 / 2x2 / 2x4 as virtual ranks, C3 as 8 virtual ranks).
#   bash tools/gpu/r4_final2.sh COMMIT -> gpurun_out/r4z/, gpurun_out/r4e/
set -o pipefail
export TMPDIR=/tmp
C=${1:-unknown}
O=gpurun_out/r4z
mkdir -p $O
rm -f gpurun_out/parity_l2.jsonl
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
cp gpurun_out/parity_l2.jsonl $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
bash tools/gpu/r4_evidence.sh $C || exit 1
for b in 2x1 2x2 2x4; do
  v=$(( ${b%x*} * ${b#*x} ))
  NLH_VIRTUAL_RANKS=$v timeout -k 10 300 python bench.py --blocks $b --steps 200 --pmc off --no-cpu-baseline > $O/weak_v${v}.json 2> $O/weak_v${v}.err || exit 1
done
NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --strong --lattice 32768 --blocks 2x4 --steps 20 --pmc off --no-cpu-baseline > $O/c3_v8.json 2> $O/c3_v8.err || exit 1
timeout -k 10 300 python -u tools/diag_sched.py 200 2x1 4096x4096 short > $O/sched_check.jsonl 2> $O/sched_check.err || exit 1
echo done > $O/done
