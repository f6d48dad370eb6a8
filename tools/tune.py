#!/usr/bin/env python3
"""A/B timing of solver configurations on one GPU, interleaved rounds in one
process (cdna_hip_programming.md 5.4 rule 24).  Each configuration is a set of
environment variables read by nlh_create (NLH_PAIR_SPLIT, NLH_PAIR, ...) plus
an optional seg_rows; per-step kernel time comes from the HIP events of
nlh_kernel_timing on the stencil stream.

    python tools/tune.py --n 4096 --eps 8 \
        --cfg '{"NLH_PAIR_SPLIT": "1"}' --cfg '{"NLH_PAIR_SPLIT": "3"}'

Prints one JSON line per configuration.
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
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--test", action="store_true")
    ap.add_argument("--kernel", default="fast")
    ap.add_argument("--cfg", action="append", default=[], help="JSON object: env vars (+ optional seg_rows)")
    a = ap.parse_args()
    n, eps = a.n, a.eps
    dh = 1.0 / n
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    cfgs = [json.loads(c) for c in a.cfg] or [{}]
    solvers = []
    base = dict(os.environ)
    for c in cfgs:
        env = {k: str(v) for k, v in c.items() if k != "seg_rows"}
        os.environ.clear()
        os.environ.update(base)
        os.environ.update(env)
        s = N.Solver(n, n, eps, 1.0, dt, dh, test=a.test, kernel=a.kernel, device=0,
                     seg_rows=int(c.get("seg_rows", 0)))
        s.test_init()
        s.run(10)
        s.synchronize()
        solvers.append((c, s))
    os.environ.clear()
    os.environ.update(base)
    res = [[] for _ in solvers]
    for _ in range(a.rounds):
        for k, (c, s) in enumerate(solvers):
            s.kernel_timing(True)
            s.run(a.steps)
            s.synchronize()
            ms, cnt = s.kernel_time()
            s.kernel_timing(False)
            res[k].append(ms / cnt * 1e3)
    for k, (c, s) in enumerate(solvers):
        us = min(res[k])
        info = s.info()
        print(json.dumps({"cfg": c, "n": n, "eps": eps, "test": a.test, "kernel": info.pass_kernel,
                          "us_per_step": us, "us_all": res[k], "gnode_s": n * n / us / 1e3}), flush=True)
        s.close()


if __name__ == "__main__":
    main()
