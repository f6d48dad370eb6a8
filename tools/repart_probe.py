"""Repartition cost probe (one GPU, virtual owners): solver creation and
explicit repartitions between two tile maps of the reference's
load_balance_25s_4n grid (5 x 5 tiles, 4 owners), with NLH_TRACE_REPART=1
phase times on stderr.  Usage: NLH_VIRTUAL_RANKS=4 NLH_TRACE_REPART=1
python tools/repart_probe.py TILE [REPS]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import nonlocalheatequation_amd as N  # noqa: E402


def main():
    tile = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    npx = npy = 5
    a = np.zeros(25, np.int32)  # the reference map: 21 tiles on owner 0
    a[[4, 9, 14, 19]] = [1, 2, 3, 1]
    b = np.arange(25, dtype=np.int32) % 4  # balanced
    n = tile * npx
    dh = 1.0 / n
    eps = 8
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    t0 = time.perf_counter()
    with N.Solver(n, n, eps, 1.0, dt, dh, tiles=(npx, npy), owner=a) as s:
        t1 = time.perf_counter()
        s.test_init()
        s.run(4)
        s.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"tile": tile, "create_ms": (t1 - t0) * 1e3, "first_4_steps_ms": (t2 - t1) * 1e3}),
              flush=True)
        for r in range(reps):
            for m in (b, a):
                t = time.perf_counter()
                s.repartition(m)
                s.synchronize()
                print(json.dumps({"tile": tile, "rep": r, "to": "balanced" if m is b else "reference",
                                  "repartition_ms": (time.perf_counter() - t) * 1e3}), flush=True)
        t = time.perf_counter()
        s.run(10)
        s.synchronize()
        print(json.dumps({"tile": tile, "ten_steps_ms": (time.perf_counter() - t) * 1e3}), flush=True)


if __name__ == "__main__":
    main()
