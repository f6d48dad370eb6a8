"""One rank's pass on one GPU (round 6): a block of the
given size alone and with the exchange-path schedule forced on chosen sides
(NLH_FORCE_BANDS side mask: 2 left, 4 right, 8 top, 16 bottom; 1 = all four),
eps 8 production, the library's default schedule.  Each case runs in a child
process (the mask is read at nlh_create), interleaved, and prints one JSON line
with the wall time per pass (two steps) over K timed steps.

  python tools/rank_proxy.py NX NY [STEPS=100] [REPS=2] [MASK ...]
"""
import json
import os
import subprocess
import sys
import time


def child(nx, ny, steps):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import nonlocalheatequation_amd as N
    eps, dh = 8, 1.0 / max(nx, ny)
    dt = eps ** 4 * dh * dh / (8.0 * N.disk_count(eps))
    with N.Solver(nx, ny, eps, 1.0, dt, dh, test=False, kernel="fast") as s:
        s.test_init()
        tw = time.perf_counter()
        while time.perf_counter() - tw < 0.5:  # the clocks a sustained run holds
            s.run(20)
            s.synchronize()
        t0 = time.perf_counter()
        s.run(steps)
        s.synchronize()
        wall = time.perf_counter() - t0
    return {"us_per_pass": wall / steps * 2e6, "gnu": nx * ny * steps / wall / 1e9}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        nx, ny, steps = (int(v) for v in sys.argv[2:5])
        print(json.dumps(child(nx, ny, steps)))
        return 0
    nx, ny = int(sys.argv[1]), int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 100
    reps = int(sys.argv[4]) if len(sys.argv) > 4 else 2
    masks = [int(m) for m in sys.argv[5:]] or [0, 1]
    for rep in range(reps):
        for m in masks:
            env = dict(os.environ)
            env.pop("NLH_FORCE_BANDS", None)
            if m:
                env["NLH_FORCE_BANDS"] = str(m)
            p = subprocess.run([sys.executable, __file__, "--child", str(nx), str(ny), str(steps)], env=env,
                               capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                print(p.stderr, file=sys.stderr)
                return p.returncode
            r = json.loads(p.stdout.strip().splitlines()[-1])
            r.update(nx=nx, ny=ny, mask=m, rep=rep + 1)
            print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
