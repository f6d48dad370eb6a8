#!/usr/bin/env python3
"""Diagnostic (GPU): the exchange-path schedule knobs (NLH_INT_PER_CU,
NLH_SCHED, NLH_COMM_PRIO, NLH_BAND_SEG; result-neutral) on a per-rank proxy
of the weak-scaling bench: one rank's 4096^2 lattice as 2x1 (or 2x2) blocks
whose halo pieces go over RCCL to self, two-step passes.  Prints wall us per
pass (best of 3 runs of P passes) per setting, and the single-block figure.

    python tools/diag_sched.py [passes=200] [tiles=2x1] [lattice=4096x4096] [full|short]
(short: NLH_SCHED=2, NLH_BAND_SEG=0, NLH_INT_PER_CU 0 / 3 / 4 x NLH_COMM_PRIO 0 / 1)"""
import itertools
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nonlocalheatequation_amd as N  # noqa: E402

PASSES = int(sys.argv[1]) if len(sys.argv) > 1 else 200
TX, TY = (int(v) for v in (sys.argv[2] if len(sys.argv) > 2 else "2x1").split("x"))
NX, NY = (int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "4096x4096").split("x"))
SHORT = len(sys.argv) > 4 and sys.argv[4] == "short"
KNOBS = ("NLH_INT_PER_CU", "NLH_SCHED", "NLH_COMM_PRIO", "NLH_BAND_SEG", "NLH_RCCL_SELF")
eps = 8
dh = 1.0 / 4096
dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))


def wall(tiles, env):
    for k in KNOBS:
        os.environ.pop(k, None)
    os.environ.update({k: str(v) for k, v in env.items()})
    with N.Solver(NX, NY, eps, 1.0, dt, dh, kernel="fast", tiles=tiles, split_tiles=True) as s:
        s.test_init()
        spp = s.info().steps_per_pass
        s.run(40)
        s.synchronize()
        best = 1e30
        for _ in range(3):
            t0 = time.perf_counter()
            s.run(PASSES * spp)
            s.synchronize()
            best = min(best, (time.perf_counter() - t0) * 1e6 / PASSES)
        return best


print(json.dumps({"setting": f"{NX}x{NY} one block", "us_per_pass": round(wall((1, 1), {}), 1)}), flush=True)
grid = (((0, 3, 4), (2,), (0, 1), (0,)) if SHORT else ((0, 2, 3, 4), (0, 1, 2), (0, 1), (0, 32)))
for ipc, sched, prio, bseg in itertools.product(*grid):
    env = {"NLH_RCCL_SELF": 1, "NLH_INT_PER_CU": ipc, "NLH_SCHED": sched, "NLH_COMM_PRIO": prio,
           "NLH_BAND_SEG": bseg}
    us = wall((TX, TY), env)
    print(json.dumps({"setting": f"{NX}x{NY} as {TX}x{TY} blocks", **{k[4:].lower(): v for k, v in env.items()},
                      "us_per_pass": round(us, 1)}), flush=True)
print("done", flush=True)
