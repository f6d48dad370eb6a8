#!/bin/bash
# Round 6: where the non-kernel time of the 20-step timed region goes
# (VERDICT r5 next 1).  tools/host_gap.py variants interleaved, two rounds:
#   poll   nlh_synchronize polls its streams (the round-6 default)
#   spin   NLH_SYNC=4: the device's spin flag + hipStreamSynchronize (round 5's default)
#   auto   NLH_SYNC=3: HIP's auto flag + hipStreamSynchronize (HIP's own default)
#   timer  poll, with a threading.Timer started right before t0 (round 5's bench)
#   probe  poll, NLH_HOST_PROBE=1 (nlh_run records when its start event completes)
# then the driver-form bench line twice, then (SUITE=1) the GPU test suite.
#   bash tools/gpu/r6_host.sh OUTDIR [REPS]
set -o pipefail
export TMPDIR=/tmp
O=${1:-gpurun_out/r6host}
REPS=${2:-100}
mkdir -p $O
for round in 1 2; do
  for v in poll spin auto timer probe; do
    env=""; extra=""
    case $v in
      spin) env="NLH_SYNC=4";;
      auto) env="NLH_SYNC=3";;
      timer) extra="--timer";;
      probe) env="NLH_HOST_PROBE=1";;
    esac
    env $env timeout -k 10 120 python tools/host_gap.py --reps $REPS --label $v $extra > $O/${v}_$round.jsonl 2> $O/${v}_$round.err || exit 1
    tail -1 $O/${v}_$round.jsonl
  done
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20_$i.json 2> $O/bench20_$i.err || exit 1
done
if [ "${SUITE:-0}" = 1 ]; then
  rm -f gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl
  timeout -k 10 1100 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log
  cp gpurun_out/parity_l2.jsonl gpurun_out/parity_nodes.jsonl $O/ 2>/dev/null
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
fi
echo done > $O/done
