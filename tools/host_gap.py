#!/usr/bin/env python3
"""Where the non-kernel time of bench.py's timed region goes.

Runs the C2 workload (4096^2, eps 8, production) in one process and repeats
bench.py's timed region -- barrier, t0, nlh_run(K), synchronize, t1 -- R
times, recording per repetition: the host wall time, nlh_run's enqueue time,
the synchronize time, the stream-event span of the passes and the library's
host timestamps (nlh_host_time: end event first seen by the polling wait;
with NLH_HOST_PROBE=1 also the start event).  The variant under test comes
from the environment (NLH_SYNC, NLH_HOST_PROBE, NLH_GRAPH,
NLH_VIRTUAL_RANKS with --blocks) and from --timer
(a threading.Timer started right before t0, as round 5's bench did).

    python tools/host_gap.py --reps 100 --steps 20 --label poll > out.jsonl

Prints one JSON record per repetition and a summary record last.
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=100)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--lattice", type=int, default=4096)
    ap.add_argument("--eps", type=int, default=8)
    ap.add_argument("--warmup-ms", type=float, default=300.0)
    ap.add_argument("--timer", action="store_true", help="start a threading.Timer right before t0")
    ap.add_argument("--label", default="")
    ap.add_argument("--blocks", default="1x1", help="PXxPY block grid over the --lattice (virtual ranks: "
                                                   "NLH_VIRTUAL_RANKS in the environment)")
    args = ap.parse_args()
    import nonlocalheatequation_amd as N
    nb, eps = args.lattice, args.eps
    dh = 1.0 / nb
    dt = eps ** 4 * dh * dh / (8.0 * N.disk_count(eps))
    px, py = (int(v) for v in args.blocks.lower().split("x"))
    s = N.Solver(nb, nb, eps, 1.0, dt, dh, test=False, kernel="fast", device=0, tiles=(px, py))
    spp = s.info().steps_per_pass
    s.test_init()
    t_end = time.perf_counter() + args.warmup_ms / 1e3
    while time.perf_counter() < t_end:
        s.run(10)
        s.synchronize()
    recs = []
    for r in range(args.reps):
        s.synchronize()
        s.kernel_timing(True)
        if args.timer:
            tm = threading.Timer(3600.0, lambda: None)
            tm.daemon = True
            tm.start()
        t0 = time.perf_counter()
        s.run(args.steps)
        t_enq = time.perf_counter()
        s.synchronize()
        t1 = time.perf_counter()
        k_ms, _ = s.kernel_time()
        h = s.host_time()
        s.kernel_timing(False)
        if args.timer:
            tm.cancel()
        wall = (t1 - t0) * 1e6
        rec = {"label": args.label, "rep": r, "wall_us": wall, "enqueue_us": (t_enq - t0) * 1e6,
               "sync_us": (t1 - t_enq) * 1e6, "span_us": k_ms * 1e3, "outside_us": wall - k_ms * 1e3,
               "lib_enqueue_us": h["enqueue_us"], "lib_start_seen_us": h["start_seen_us"],
               "lib_end_seen_us": h["end_seen_us"], "lib_sync_return_us": h["sync_return_us"],
               "lib_enqueue_us_per_pass": h["enqueue_us"] / max(1, args.steps // spp)}
        if h["end_seen_us"] >= 0 and h["sync_return_us"] >= 0:
            rec["tail_us"] = h["sync_return_us"] - h["end_seen_us"]
            # host-side estimate of the GPU's start: end seen minus the span
            rec["head_us"] = h["end_seen_us"] - k_ms * 1e3
        recs.append(rec)
        print(json.dumps(rec), flush=True)
    summ = {"label": args.label, "summary": True, "reps": args.reps, "steps": args.steps,
            "env": {k: os.environ.get(k) for k in ("NLH_SYNC", "NLH_HOST_PROBE", "NLH_GRAPH", "NLH_VIRTUAL_RANKS")},
            "timer": args.timer, "build_id": N.build_id(), "blocks": args.blocks, "lattice": nb,
            "virtual_ranks": os.environ.get("NLH_VIRTUAL_RANKS")}
    for k in ("wall_us", "outside_us", "enqueue_us", "sync_us", "span_us", "tail_us", "head_us",
              "lib_enqueue_us_per_pass"):
        v = [x[k] for x in recs if k in x]
        if v:
            summ[k] = {"median": statistics.median(v), "p10": pct(v, 0.1), "p90": pct(v, 0.9), "max": max(v),
                       "min": min(v)}
    summ["gnu_median"] = nb * nb * args.steps / (summ["wall_us"]["median"] * 1e-6) / 1e9
    print(json.dumps(summ), flush=True)
    s.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
