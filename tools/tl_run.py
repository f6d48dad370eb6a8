#!/usr/bin/env python3
"""Short stepping program for a rocprofv3 kernel timeline of the multi-block
schedule: NLH_* env as set by the caller; tiles/split from argv."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nonlocalheatequation_amd as N  # noqa: E402

n = int(os.environ.get("NLH_N", "4096"))
tx, ty = int(sys.argv[1]), int(sys.argv[2])
split = len(sys.argv) > 3 and sys.argv[3] == "split"
eps = 8
dh = 1.0 / n
dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
with N.Solver(n, n, eps, 1.0, dt, dh, test=False, kernel="fast", device=0, tiles=(tx, ty), split_tiles=split) as s:
    s.test_init()
    s.run(40)
    s.synchronize()
print("ok")
