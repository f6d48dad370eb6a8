#!/usr/bin/env python3
"""Minimal C2 stepping program for rocprofv3 --pmc passes (no CPU baseline,
no torch): 4096^2, eps=8, fast kernel, 10 warm-up + N timed steps."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nonlocalheatequation_amd as N  # noqa: E402

n = int(os.environ.get("NLH_N", "4096"))
eps = int(os.environ.get("NLH_EPS", "8"))
steps = int(os.environ.get("NLH_STEPS", "20"))
kernel = os.environ.get("NLH_KERNEL", "fast")
dh = 1.0 / n
dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
s = N.Solver(n, n, eps, 1.0, dt, dh, test=False, kernel=kernel, device=0,
             seg_rows=int(os.environ.get("NLH_SEG", "0")))
s.test_init()
s.run(10 + steps)
s.synchronize()
s.close()
print("ok")
