#!/bin/bash
# Round 5, call Q (the cost of --nbalance's busy timing): the
# distributed driver on 4 virtual owners, 4096^2 tiles, eps 8, 400 steps
#   balanced 2x2 map (one tile per owner): no balancing / --nbalance 100
#   (busy window of 26 steps per interval) / --nbalance 100 --test_load_balance
#   (busy timing throughout); the reference's 25-tile map load_balance_25s_4n
#   at 1024^2 tiles: no balancing / --nbalance 50
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
python3 - <<'PY' || exit 1
import nonlocalheatequation_amd as N
n = 8192; dh = 1.0 / n
open("gpurun_out/r5q/bal.txt", "w").write(f"4096 4096 2 2 {dh}\n0 0 0\n1 0 1\n0 1 2\n1 1 3\n")
open("gpurun_out/r5q/dt", "w").write(repr(8 ** 4 * dh * dh / (8 * N.disk_count(8))))
src = [l.split() for l in open("tests/golden/reference_inputs/load_balance_25s_4n.txt").read().split("\n") if l.strip()]
npx, npy = int(src[0][2]), int(src[0][3])
m = 1024 * npx; dh2 = 1.0 / m
lines = [f"1024 1024 {npx} {npy} {dh2}"] + [" ".join(r[:3]) for r in src[1:]]
open("gpurun_out/r5q/lb25.txt", "w").write("\n".join(lines) + "\n")
open("gpurun_out/r5q/dt25", "w").write(repr(8 ** 4 * dh2 * dh2 / (8 * N.disk_count(8))))
PY
DT=$(cat $O/dt); DT25=$(cat $O/dt25)
D=bin/2d_nonlocal_distributed
for rep in 1 2; do
  NLH_VIRTUAL_RANKS=4 timeout -k 10 200 $D --file $O/bal.txt --nt 400 --dt $DT --eps 8 --nlog 100000 > $O/bal_none_$rep.log 2>&1 || exit 1
  NLH_VIRTUAL_RANKS=4 timeout -k 10 200 $D --file $O/bal.txt --nt 400 --dt $DT --eps 8 --nlog 100000 --nbalance 100 > $O/bal_nb100_$rep.log 2>&1 || exit 1
  NLH_VIRTUAL_RANKS=4 timeout -k 10 200 $D --file $O/bal.txt --nt 400 --dt $DT --eps 8 --nlog 100000 --nbalance 100 --test_load_balance > $O/bal_nb100_lbt_$rep.log 2>&1 || exit 1
  NLH_VIRTUAL_RANKS=4 timeout -k 10 200 $D --file $O/lb25.txt --nt 400 --dt $DT25 --eps 8 --nlog 100000 > $O/lb25_none_$rep.log 2>&1 || exit 1
  NLH_VIRTUAL_RANKS=4 timeout -k 10 200 $D --file $O/lb25.txt --nt 400 --dt $DT25 --eps 8 --nlog 100000 --nbalance 50 > $O/lb25_nb50_$rep.log 2>&1 || exit 1
done
echo done > $O/done
