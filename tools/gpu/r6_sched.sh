set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r6sched; mkdir -p $O
# C2-size rank proxies by mask and schedule
bash tools/gpu/r6_band_sched.sh $O/c2 "m4s2:NLH_FORCE_BANDS=4" "m4s0:NLH_FORCE_BANDS=4,NLH_SCHED=0" "m26s2:NLH_FORCE_BANDS=26" "m26s0:NLH_FORCE_BANDS=26,NLH_SCHED=0" "m30s2:NLH_FORCE_BANDS=30" "m30s0:NLH_FORCE_BANDS=30,NLH_SCHED=0" "m30s1:NLH_FORCE_BANDS=30,NLH_SCHED=1" || exit 1
# virtual-rank lines with real RCCL-to-self messages
for sc in 2 0; do
  NLH_SCHED=$sc NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --strong --lattice 32768 --blocks 2x4 --steps 20 --pmc off --no-cpu-baseline > $O/c3v8_s$sc.json 2> $O/c3v8_s$sc.err || exit 1
  NLH_SCHED=$sc NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --blocks 2x4 --steps 200 --pmc off --no-cpu-baseline > $O/weakv8_s$sc.json 2> $O/weakv8_s$sc.err || exit 1
  NLH_SCHED=$sc NLH_VIRTUAL_RANKS=2 timeout -k 10 300 python bench.py --blocks 2x1 --steps 200 --pmc off --no-cpu-baseline > $O/weakv2_s$sc.json 2> $O/weakv2_s$sc.err || exit 1
  for f in c3v8 weakv8 weakv2; do python3 -c "import json; d=json.load(open('$O/${f}_s$sc.json')); print('${f}_s$sc', round(d['value'],1), d.get('exchange',{}).get('exposed_share_of_pass'))"; done
done
