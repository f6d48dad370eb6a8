set -u
# fresh-container re-check: whole GPU suite, smoke, bench evidence
O=gpurun_out/s3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
tools/bench_evidence.sh s3/ev k_pair_split || exit 1
cat $O/ev/bench.json
echo done
