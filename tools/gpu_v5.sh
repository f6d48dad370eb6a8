set -u
O=gpurun_out/v5
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo pytest failed; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
tools/bench_evidence.sh v5/ev k_pair_split || exit 1
NLH_PAIR_ABLATE=1207 tools/pmc.sh $O/pmc_nohbm > $O/pmc_nohbm.log 2>&1 || exit 1
python tools/pmc_summary.py $O/pmc_nohbm k_pair_split > $O/pmc_nohbm_summary.json || exit 1
echo done
