#!/usr/bin/env python3
"""Generate the field fixtures under tests/golden/ from the CPU oracle.

The oracle (oracle/nlh_oracle.c) is pinned bit-for-bit against the
reference's own outputs recorded in tests/golden/known_answers.json (SURVEY.md
Appendix A), see tests/test_oracle.py.  These fixtures freeze its final fields
so that GPU parity can also be checked against stored data:

  fields_2d_row{0,5,7}_test{0,1}.npy   tests/2d.txt rows 0, 5, 7 (50^2, 40^2, 40^2)
  field_eps32_96_test{0,1}.npy         96^2, eps=32, 2 steps, dh=1/96, dt rule
  l2_per_step_row0.npy                 error_l2 at t = 1..45 for tests/2d.txt row 0

Run from the repository root:  python tools/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

ROWS = {0: (50, 50, 45, 5, 1.0, 0.0005, 0.02),
        5: (40, 40, 200, 3, 0.2, 0.001, 0.02),
        7: (40, 40, 200, 8, 0.2, 0.001, 0.02)}


def n_disk(eps):
    return O.disk_count(eps)


def main():
    for r, (nx, ny, nt, eps, k, dt, dh) in ROWS.items():
        for test in (0, 1):
            p = O.params(nx, ny, eps, k, dt, dh, test)
            u = O.run(p, nt)
            np.save(os.path.join(OUT, f"fields_2d_row{r}_test{test}.npy"), u)
    nx = 96
    dh = 1.0 / nx
    dt = 32 ** 4 * dh * dh / (8 * 1.0 * n_disk(32))
    for test in (0, 1):
        p = O.params(nx, nx, 32, 1.0, dt, dh, test)
        np.save(os.path.join(OUT, f"field_eps32_96_test{test}.npy"), O.run(p, 2))
    nx, ny, nt, eps, k, dt, dh = ROWS[0]
    p = O.params(nx, ny, eps, k, dt, dh, 1)
    u = O.test_init(p)
    l2 = []
    for t in range(nt):
        u = O.step(p, t, u)
        l2.append(O.errors(p, t + 1, u)[0])
    np.save(os.path.join(OUT, "l2_per_step_row0.npy"), np.array(l2))
    print("fixtures written to", OUT)


if __name__ == "__main__":
    main()
