#!/usr/bin/env python3
"""One-GPU rehearsal of the multi-GPU step schedule: wall time
per step of the production path for
  single     one block, no exchange
  bands      one block through the exchange schedule (NLH_FORCE_BANDS)
  local TxT  TxT tiles as separate blocks, halo pieces by device copies
  rccl TxT   the same, pieces packed and sent over RCCL send/recv to self
             (NLH_RCCL_SELF) -- the multi-GPU transport and its overlap
One JSON line per configuration.
    python tools/sched_probe.py [--nx 4096] [--ny 4096] [--eps 8] [--steps 200]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import nonlocalheatequation_amd as N  # noqa: E402


def timed(nx, ny, eps, steps, rounds, tiles=(1, 1), split=False, env=None):
    env = env or {}
    for k, v in env.items():
        os.environ[k] = v
    try:
        dh = 1.0 / nx
        dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
        with N.Solver(nx, ny, eps, 1.0, dt, dh, test=False, kernel="fast", device=0,
                      tiles=tiles, split_tiles=split) as s:
            s.test_init()
            s.run(10)
            s.synchronize()
            best = None
            for _ in range(rounds):
                t0 = time.perf_counter()
                s.run(steps)
                s.synchronize()
                us = (time.perf_counter() - t0) / steps * 1e6
                best = us if best is None else min(best, us)
            info = s.info()
            return {"us_per_step": best, "gnode_s": nx * ny / best / 1e3, "nblocks": info.nblocks,
                    "npeers": info.npeers, "halo_bytes_per_pass": info.halo_bytes_sent,
                    "kernel": info.pass_kernel}
    finally:
        for k in env:
            os.environ.pop(k, None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=4096)
    ap.add_argument("--ny", type=int, default=4096)
    ap.add_argument("--eps", type=int, default=8)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--tiles", default="2x2,4x2")
    ap.add_argument("--no-single", action="store_true")
    a = ap.parse_args()
    base = {"nx": a.nx, "ny": a.ny, "eps": a.eps,
            "env": {k: v for k, v in os.environ.items() if k in ("NLH_SCHED", "NLH_INT_PER_CU", "NLH_BAND_SEG", "NLH_COMM_PRIO")}}
    cfgs = [] if a.no_single else [("single", {}, (1, 1), False)]
    cfgs.append(("bands", {"NLH_FORCE_BANDS": "1"}, (1, 1), False))
    for t in a.tiles.split(","):
        tx, ty = map(int, t.split("x"))
        cfgs.append((f"local {t}", {}, (tx, ty), True))
        cfgs.append((f"rccl {t}", {"NLH_RCCL_SELF": "1"}, (tx, ty), True))
    for name, env, tiles, split in cfgs:
        r = timed(a.nx, a.ny, a.eps, a.steps, a.rounds, tiles, split, env)
        print(json.dumps({"config": name, **base, **r}), flush=True)


if __name__ == "__main__":
    main()
