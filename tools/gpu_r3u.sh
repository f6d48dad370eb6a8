set -o pipefail
# round 3, re-entry: row-pair k_pair_split harness vs the round-3 kernel, then
# GPU suite + smoke + bench at the rebuilt HEAD, then the shader clock the
# fp64 kernels actually run at (GRBM_GUI_ACTIVE cycles per kernel duration;
# rocm-smi samples during a long bench run).  Stops after any step that ends
# in a fault, abort or time limit (exit status other than 0 / 1).
export TMPDIR=/tmp
O=gpurun_out/r3u
mkdir -p $O
timeout -k 10 200 ./build/pair_bench 4096 200 > $O/pair_rows.jsonl 2> $O/pair_rows.err
rc=$?; echo "pair_bench rc=$rc" >> $O/pair_rows.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err && \
NLH_N=4096 NLH_EPS=8 NLH_STEPS=1000 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace \
  --output-format csv -d $O/clk_c2 -o run -- python tools/prof_step.py > $O/clk_c2.log 2>&1 && \
NLH_N=8192 NLH_EPS=32 NLH_STEPS=400 timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace \
  --output-format csv -d $O/clk_c4 -o run -- python tools/prof_step.py > $O/clk_c4.log 2>&1 && \
python tools/smi_during.py $O/smi_c2.jsonl -- timeout -k 10 120 python bench.py --steps 200000 --warmup 5 \
  --pmc off --no-cpu-baseline > $O/smi_c2_bench.json 2> $O/smi_c2_bench.err
rc=$?; echo "done rc=$rc" >> $O/smoke.log; exit $rc
