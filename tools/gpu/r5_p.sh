#!/bin/bash
# Round 5, call P: NLH_PAIR_PRIO on the exchange layouts -- C3 as 2x4 virtual
# ranks and the weak 2x4 layout, wave priority auto (1), never (0), not on the
# edge bands (2), each twice, interleaved
set -o pipefail
O=gpurun_out/r5p
mkdir -p $O
for rep in 1 2; do
  for pp in 1 0 2; do
    NLH_PAIR_PRIO=$pp NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --strong --lattice 32768 --blocks 2x4 --steps 20 --pmc off --no-cpu-baseline > $O/c3_v8_p${pp}_$rep.json 2> $O/c3_v8_p${pp}_$rep.err || exit 1
    NLH_PAIR_PRIO=$pp NLH_VIRTUAL_RANKS=8 timeout -k 10 300 python bench.py --blocks 2x4 --steps 200 --pmc off --no-cpu-baseline > $O/weak_v8_p${pp}_$rep.json 2> $O/weak_v8_p${pp}_$rep.err || exit 1
  done
done
echo done > $O/done
