set -u
# exchange-schedule sweep at 4096^2 (one GPU; RCCL self transport), then timelines
O=gpurun_out/s7
mkdir -p $O
export TMPDIR=/tmp
run() { timeout -k 10 200 env "$@" python -u tools/sched_probe.py --nx 4096 --ny 4096 --tiles 2x2 --no-single --rounds 5 >> $O/sched.jsonl 2>> $O/sched.err || { echo "failed: $*"; tail $O/sched.err; exit 1; }; }
timeout -k 10 100 python -u tools/sched_probe.py --tiles 2x2 --rounds 5 --no-single > /dev/null 2>&1
run NLH_SCHED=0
run NLH_SCHED=0 NLH_INT_PER_CU=3
run NLH_SCHED=2
run NLH_SCHED=2 NLH_INT_PER_CU=3
run NLH_SCHED=2 NLH_INT_PER_CU=3 NLH_COMM_PRIO=1
run NLH_SCHED=2 NLH_INT_PER_CU=3 NLH_BAND_SEG=16
run NLH_SCHED=2 NLH_INT_PER_CU=3 NLH_BAND_SEG=64
run NLH_SCHED=0 NLH_INT_PER_CU=3 NLH_COMM_PRIO=1
NLH_SCHED=2 NLH_INT_PER_CU=3 NLH_RCCL_SELF=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/rccl2 -o run -- python3 tools/tl_run.py 2 2 split > $O/rccl2.log 2>&1 || { echo tl failed; exit 1; }
python tools/timeline.py $O/rccl2/run_kernel_trace.csv --last 24 > $O/rccl2_timeline.txt
cat $O/rccl2_timeline.txt
echo done
