set -u
# schedule variants of the multi-block step at 4096^2 (one GPU, RCCL self transport)
O=gpurun_out/s5
mkdir -p $O
run() { timeout -k 10 200 env "$@" python -u tools/sched_probe.py --nx 4096 --ny 4096 --tiles 2x2,4x2 --no-single >> $O/sched.jsonl 2>> $O/sched.err || { echo "failed: $*"; tail $O/sched.err; exit 1; }; }
run NLH_SCHED=0
run NLH_SCHED=1
run NLH_SCHED=0 NLH_INT_PER_CU=3
run NLH_SCHED=1 NLH_INT_PER_CU=3
run NLH_SCHED=0 NLH_INT_PER_CU=2
cat $O/sched.jsonl
echo done
