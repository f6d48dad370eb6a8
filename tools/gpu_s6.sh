set -u
# kernel timelines of the exchange schedule at 4096^2 (bands on one block; RCCL self 2x2)
O=gpurun_out/s6
mkdir -p $O
export TMPDIR=/tmp
NLH_FORCE_BANDS=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/bands -o run -- python3 tools/tl_run.py 1 1 > $O/bands.log 2>&1 || { echo bands failed; tail $O/bands.log; exit 1; }
NLH_RCCL_SELF=1 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/rccl -o run -- python3 tools/tl_run.py 2 2 split > $O/rccl.log 2>&1 || { echo rccl failed; tail $O/rccl.log; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/single -o run -- python3 tools/tl_run.py 1 1 > $O/single.log 2>&1 || { echo single failed; tail $O/single.log; exit 1; }
echo done
