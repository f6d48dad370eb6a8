set -u
# multi-GPU schedule rehearsal on one GPU (RCCL self transport) + secondary bench lines
O=gpurun_out/s4
mkdir -p $O
timeout -k 10 300 python -u tools/sched_probe.py --nx 4096 --ny 4096 --tiles 2x2,4x2 > $O/sched_4096.jsonl 2> $O/sched_4096.err || { echo sched4096 failed; tail $O/sched_4096.err; exit 1; }
cat $O/sched_4096.jsonl
timeout -k 10 300 python -u tools/sched_probe.py --nx 16384 --ny 8192 --steps 40 --tiles 2x1 > $O/sched_c3share.jsonl 2> $O/sched_c3share.err || { echo sched c3 failed; tail $O/sched_c3share.err; exit 1; }
cat $O/sched_c3share.jsonl
timeout -k 10 300 python bench.py --eps 32 --lattice 8192 --steps 40 --warmup 4 > $O/bench_c4.json 2> $O/bench_c4.err || { echo c4 failed; tail $O/bench_c4.err; exit 1; }
cat $O/bench_c4.json
timeout -k 10 300 python bench.py --test-mode --steps 200 --warmup 10 > $O/bench_test_fast.json 2> $O/bench_test_fast.err || { echo testmode failed; tail $O/bench_test_fast.err; exit 1; }
cat $O/bench_test_fast.json
timeout -k 10 300 python bench.py --lattice 32768 --strong --steps 40 --warmup 4 --no-cpu-baseline > $O/bench_c3_1gpu.json 2> $O/bench_c3_1gpu.err || { echo c3 failed; tail $O/bench_c3_1gpu.err; exit 1; }
cat $O/bench_c3_1gpu.json
echo done
