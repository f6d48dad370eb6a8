#!/usr/bin/env python3
"""Diagnostic (GPU): where does the virtual-rank busy-timing run of
tests/test_gpu_balance.py::test_virtual_busy_measured_per_rank diverge from
the single-block run?  Each case runs the 4 x 4 tile map (1 / 5 / 4 / 6 tiles)
over NLH_VIRTUAL_RANKS=4 and compares with one block after the same steps;
prints max |diff| / field scale and the first bad row / column.

    python tools/diag_busy.py TILE   (e.g. 2048, 4096, 8192)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nonlocalheatequation_amd as N  # noqa: E402

TILE = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
T = 4
OWN = np.array([0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3], np.int32)
nx = ny = T * TILE
eps = 8
dh = 1.0 / nx
dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))


def reference(steps):
    os.environ.pop("NLH_VIRTUAL_RANKS", None)
    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="fast") as r:
        r.test_init()
        r.run(steps)
        return r.field()


def report(name, u, ref):
    d = np.abs(u - ref)
    m = float(d.max())
    scale = float(np.abs(ref).max())
    bad = np.argwhere(d > 1e-12 * scale)
    where = ""
    if len(bad):
        y0, x0 = bad.min(axis=0)
        y1, x1 = bad.max(axis=0)
        where = f" bad rows {y0}..{y1} cols {x0}..{x1} ({len(bad)} nodes)"
    print(f"{name:40s} max|diff|/scale = {m / scale:.3e}{where}", flush=True)


EVEN = np.array([0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3], np.int32)


def virtual(prog):
    """prog: list of ("timing", mode) / ("run", n) / ("move", map) /
    ("rebalance", None)."""
    os.environ["NLH_VIRTUAL_RANKS"] = "4"
    own = M7 if prog[0][0] == "start" else OWN
    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="fast", tiles=(T, T), owner=own) as s:
        s.test_init()
        for op, a in prog:
            if op == "start":
                continue
            if op == "timing":
                s.kernel_timing(a)
            elif op == "run":
                s.run(a)
            elif op == "move":
                s.repartition(a)
            else:
                s.synchronize()
                m, cur, busy = s.rebalance()
                print(f"   rebalance moved {m}: {cur.tolist()} busy {np.round(busy, 2).tolist()}",
                      flush=True)
        s.synchronize()
        return s.field(), s.step_index


CASES = [
    ("timing 0, 10", [("run", 10)]),
    ("timing 2, 10", [("timing", 2), ("run", 10)]),
    ("timing 2, 11", [("timing", 2), ("run", 11)]),
    ("timing 3, 10", [("timing", 3), ("run", 10)]),
    ("run 4, timing 2, run 6", [("run", 4), ("timing", 2), ("run", 6)]),
    ("timing 0, move after 4, +6", [("run", 4), ("move", EVEN), ("run", 6)]),
    ("timing 2, move after 4, +6", [("timing", 2), ("run", 4), ("move", EVEN), ("run", 6)]),
    ("run 4, timing 2, run 20, rebalance, run 6",
     [("run", 4), ("timing", 2), ("run", 20), ("rebalance", None), ("run", 6)]),
    ("run 4, move to M7 (no steps after)", [("run", 4), ("move", None)]),
    ("run 4, move to M7, run 6", [("run", 4), ("move", None), ("run", 6)]),
    ("timing 2, run 4, move to M7, run 6", [("timing", 2), ("run", 4), ("move", None), ("run", 6)]),
    ("run 24, move to M7, run 6", [("run", 24), ("move", None), ("run", 6)]),
    ("M7 from the start, run 6", [("start", None), ("run", 6)]),
]
# the map case 7's rebalance chose on 8192^2 tiles (profiles/r04/fifth)
M7 = np.array([0, 1, 1, 1, 0, 1, 2, 2, 2, 2, 3, 3, 0, 3, 3, 3], np.int32)
CASES = [(n, [(op, M7 if op == "move" and a is None else a) for op, a in p]) for n, p in CASES]
only = sys.argv[2:] and set(int(a) for a in sys.argv[2:])
for i, (name, prog) in enumerate(CASES):
    if only and i not in only:
        continue
    u, t = virtual(prog)
    report(f"[{i}] {name} (t={t})", u, reference(t))
    del u
print("done", flush=True)
