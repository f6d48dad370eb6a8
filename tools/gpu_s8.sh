set -u
# new exchange-schedule defaults: multiblock parity, then probes at 4096^2 and the C3 per-GPU share
O=gpurun_out/s8
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multiblock.py tests/test_drivers.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/sched_probe.py --nx 4096 --ny 4096 --tiles 2x2,4x2 --rounds 5 > $O/sched_4096.jsonl 2> $O/sched_4096.err || { echo probe failed; exit 1; }
timeout -k 10 300 python -u tools/sched_probe.py --nx 16384 --ny 8192 --steps 40 --tiles 2x1 --rounds 3 > $O/sched_c3share.jsonl 2> $O/sched_c3share.err || { echo probe c3 failed; exit 1; }
NLH_INT_PER_CU=0 timeout -k 10 300 python -u tools/sched_probe.py --nx 16384 --ny 8192 --steps 40 --tiles 2x1 --rounds 3 --no-single >> $O/sched_c3share.jsonl 2>> $O/sched_c3share.err || { echo probe c3b failed; exit 1; }
grep -h '^{' $O/*.jsonl
echo done
