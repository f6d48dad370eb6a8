#!/usr/bin/env python3
"""Per-horizon comparison of the production paths on one GPU: the two-step
pass k_pair (NLH_PAIR=1) against the single-step k_fast (NLH_PAIR=0), per
time step, HIP events on the stencil stream.  One JSON line per eps.
    python tools/tune_eps.py [--n 4096] [--eps 1-16] [--steps 40]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import nonlocalheatequation_amd as N  # noqa: E402


def parse_eps(s):
    out = []
    for part in s.split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--eps", default="1-16")
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    n = a.n
    dh = 1.0 / n
    for eps in parse_eps(a.eps):
        dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
        row = {"eps": eps, "n": n}
        for pair in (1, 0):
            os.environ["NLH_PAIR"] = str(pair)
            s = N.Solver(n, n, eps, 1.0, dt, dh, test=False, kernel="fast", device=0)
            s.test_init()
            s.run(4)
            s.synchronize()
            best = None
            for _ in range(a.rounds):
                s.kernel_timing(True)
                s.run(a.steps)
                s.synchronize()
                ms, cnt = s.kernel_time()
                s.kernel_timing(False)
                us = ms / cnt * 1e3
                best = us if best is None else min(best, us)
            row["pair" if pair else "fast"] = {"us_per_step": best, "gnode_s": n * n / best / 1e3,
                                              "steps_per_pass": s.info().steps_per_pass}
            s.close()
        print(json.dumps(row), flush=True)
    os.environ.pop("NLH_PAIR", None)


if __name__ == "__main__":
    main()
