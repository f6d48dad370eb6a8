#!/usr/bin/env python3
"""Diagnostic (GPU): host enqueue time of nlh_run per pass against the GPU
time per pass, for the layouts of the multi-GPU bench.  If the host needs
about as long to enqueue a pass (stencil launches, events, pack / grouped
ncclSend+ncclRecv / unpack) as the GPU needs to run it, a real rank on its
own GPU would be host-bound.

    python tools/diag_enqueue.py [passes=20]

Prints one JSON line per layout: enqueue_us_per_pass (nlh_run's return),
wall_us_per_pass (after synchronize), owners (virtual ranks)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import nonlocalheatequation_amd as N  # noqa: E402

PASSES = int(sys.argv[1]) if len(sys.argv) > 1 else 20
eps = 8


def measure(name, nx, ny, tiles=(1, 1), env=None, **kw):
    for k in ("NLH_VIRTUAL_RANKS", "NLH_RCCL_SELF"):
        os.environ.pop(k, None)
    os.environ.update(env or {})
    dh = 1.0 / 4096
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="fast", tiles=tiles, **kw) as s:
        s.test_init()
        spp = s.info().steps_per_pass
        s.run(40)
        s.synchronize()
        best = None
        for _ in range(3):
            t0 = time.perf_counter()
            s.run(PASSES * spp)
            t1 = time.perf_counter()
            s.synchronize()
            t2 = time.perf_counter()
            r = ((t1 - t0) * 1e6 / PASSES, (t2 - t0) * 1e6 / PASSES)
            best = r if best is None or r[1] < best[1] else best
        info = s.info()
        print(json.dumps({"layout": name, "owners": info.owners, "blocks": info.nblocks,
                          "enqueue_us_per_pass": round(best[0], 1), "wall_us_per_pass": round(best[1], 1),
                          "enqueue_us_per_pass_per_owner": round(best[0] / max(1, info.owners), 1)}), flush=True)


measure("4096^2 one block", 4096, 4096)
measure("4096^2 one rank, 2x1 blocks over RCCL to self", 4096, 4096, tiles=(2, 1), split_tiles=True,
        env={"NLH_RCCL_SELF": "1"})
measure("4096^2 one rank, 2x2 blocks over RCCL to self", 4096, 4096, tiles=(2, 2), split_tiles=True,
        env={"NLH_RCCL_SELF": "1"})
measure("weak 2x4: 8 virtual ranks of 4096^2", 2 * 4096, 4 * 4096, tiles=(2, 4), env={"NLH_VIRTUAL_RANKS": "8"})
print("done", flush=True)
