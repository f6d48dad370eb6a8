#!/usr/bin/env python3
"""Sweep the fast kernels' segment height on the C2 workload (4096^2, eps=8)
and report per-launch kernel time from HIP events, interleaved rounds in one
process (cdna_hip_programming.md 5.4 rule 24).  Usage:
    python tools/tune_fast.py [--eps 8] [--n 4096] [--segs 32,64,128,256]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import nonlocalheatequation_amd as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--eps", type=int, default=8)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--segs", default="32,48,64,96,128,192,256")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--test", action="store_true")
    ap.add_argument("--rs", default="2", help="comma list of columns-per-lane variants (1,2,4)")
    ap.add_argument("--pair", default="1", help="comma list: 1 = two-step pass (k_pair), 0 = k_fast only")
    ap.add_argument("--pads", default="0", help="comma list of NLH_PITCH_PAD values (doubles)")
    ap.add_argument("--pair-ablate", default="", help="comma list of NLH_PAIR_ABLATE masks (pair=1 rows)")
    ap.add_argument("--ablate", default="0", help="comma list of NLH_ABLATE codes (100*variant + D; variant 0 prod, 1 no math, 2 no HBM)")
    a = ap.parse_args()
    n, eps = a.n, a.eps
    dh = 1.0 / n
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    segs = [int(s) for s in a.segs.split(",")]
    solvers = {}
    modes = [int(v) for v in a.pair.split(",")] + [-int(v) for v in a.ablate.split(",") if v]
    modes += [1000 + int(v) for v in a.pair_ablate.split(",") if v]
    for f2 in modes:
        os.environ["NLH_PAIR"] = str(1 if f2 >= 1000 else max(f2, 0))
        os.environ["NLH_ABLATE"] = str(max(-f2, 0))
        os.environ["NLH_PAIR_ABLATE"] = str(f2 - 1000 if f2 >= 1000 else 0)
        for r in [int(v) for v in a.rs.split(",")]:
            os.environ["NLH_FAST_R"] = str(r)
            for pad in [int(v) for v in a.pads.split(",")]:
                os.environ["NLH_PITCH_PAD"] = str(pad)
                for sg in segs:
                    s = N.Solver(n, n, eps, 1.0, dt, dh, test=a.test, kernel="fast", device=0, seg_rows=sg)
                    s.test_init()
                    s.run(10)
                    s.synchronize()
                    solvers[(f2, r, sg, pad)] = s
    segs = list(solvers)
    res = {sg: [] for sg in segs}
    for _ in range(a.rounds):
        for sg, s in solvers.items():
            s.kernel_timing(True)
            s.run(a.steps)
            s.synchronize()
            ms, cnt = s.kernel_time()
            s.kernel_timing(False)
            res[sg].append(ms / cnt * 1e3)
    out = []
    for sg in segs:
        us = min(res[sg])
        out.append({"pair": sg[0], "r": sg[1], "seg_rows": sg[2], "pad": sg[3], "us_min": us, "us_all": res[sg],
                    "gnode_s": n * n / us / 1e3, "gb_s": 16 * n * n / us / 1e3})
    print(json.dumps({"eps": eps, "n": n, "test": a.test, "results": out}))


if __name__ == "__main__":
    main()
