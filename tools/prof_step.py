#!/usr/bin/env python3
"""Minimal stepping program for rocprofv3 passes (no CPU baseline, no torch):
the bench.py workload selected by environment variables --
NLH_N (lattice edge, 4096), NLH_EPS (8), NLH_TEST (0/1), NLH_KERNEL (fast),
NLH_INFLUENCE (constant), NLH_STEPS (20 timed after 10 warm-up), NLH_SEG
(0 = automatic).  Prints one line: ok <pass kernel> <steps per pass>
<nodes> <build id>."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nonlocalheatequation_amd as N  # noqa: E402

n = int(os.environ.get("NLH_N", "4096"))
eps = int(os.environ.get("NLH_EPS", "8"))
steps = int(os.environ.get("NLH_STEPS", "20"))
kernel = os.environ.get("NLH_KERNEL", "fast")
influence = os.environ.get("NLH_INFLUENCE", "constant")
test = os.environ.get("NLH_TEST", "0") == "1"
dh = 1.0 / n
dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
if influence == "linear":
    dt /= 5.0  # as bench.py
s = N.Solver(n, n, eps, 1.0, dt, dh, test=test, kernel=kernel, device=0, influence=influence,
             seg_rows=int(os.environ.get("NLH_SEG", "0")))
s.test_init()
s.run(10 + steps)
s.synchronize()
info = s.info()
s.close()
print(f"ok {info.pass_kernel} {info.steps_per_pass} {info.owned_nodes} {N.build_id()}")
