set -u
# interior residency with an exchange: 4 blocks of 4096^2 (8192^2 split 2x2, RCCL self) -- the per-GPU block of the weak-scaling bench
O=gpurun_out/s9
mkdir -p $O
for ipc in 3 0 3 0; do
NLH_INT_PER_CU=$ipc timeout -k 10 300 python -u tools/sched_probe.py --nx 8192 --ny 8192 --steps 100 --tiles 2x2 --rounds 3 > $O/p$ipc.jsonl 2> $O/p$ipc.err || { echo probe failed; exit 1; }
grep -h '^{' $O/p$ipc.jsonl | cut -c1-160
done
echo done
