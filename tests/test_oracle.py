"""CPU: pin the oracle (oracle/nlh_oracle.c) against the reference's outputs.

known_answers.json holds the reference serial solver's own outputs (SURVEY.md
Appendix A).  The oracle must reproduce them bit for bit; the tiled restatement
of 2d_nonlocal_async must equal the serial one bit for bit; and the reference's
batch contract (error_l2 / N <= 1e-6, CMakeLists.txt:101-154) must hold on all
three batch files.
"""
import json
import os

import numpy as np
import pytest

from conftest import ROOT, read_input

import nonlocalheatequation_amd as N

KA = json.load(open(os.path.join(ROOT, "tests", "golden", "known_answers.json")))
GOLD = os.path.join(ROOT, "tests", "golden")


def _seq_sum(u):
    s = 0.0
    for v in u.ravel():  # storage order, sequential (as the survey summed)
        s += float(v)
    return s


@pytest.mark.parametrize("i", range(len(KA["serial_2d_txt"])))
def test_oracle_matches_reference_serial(oracle, i):
    a = KA["serial_2d_txt"][i]
    p = oracle.params(a["nx"], a["ny"], a["eps"], a["k"], a["dt"], a["dh"], 1)
    u = oracle.run(p, a["nt"])
    l2, li = oracle.errors(p, a["nt"], u)
    assert l2 == a["l2"]
    assert li == a["linf"]
    assert float(u[1, 1]) == a["u_1_1"]
    if a["nx"] * a["ny"] <= 2500:
        assert _seq_sum(u) == a["sum_u"]


@pytest.mark.parametrize("i", range(len(KA["tiled_rows_global"])))
def test_oracle_matches_reference_tiled_rows(oracle, i):
    a = KA["tiled_rows_global"][i]
    p = oracle.params(a["nx"], a["ny"], a["eps"], a["k"], a["dt"], a["dh"], 1)
    u = oracle.run(p, a["nt"])
    l2, li = oracle.errors(p, a["nt"], u)
    assert l2 == a["l2"]
    assert li == a["linf"]


@pytest.mark.parametrize("fmt,name", [("serial", "2d.txt"), ("async", "2d_async.txt"),
                                      ("distributed", "2d_distributed.txt")])
def test_reference_batch_contract(oracle, fmt, name):
    for r in N.parse_batch(read_input(name), fmt):
        p = oracle.params(r.nx, r.ny, r.eps, r.k, r.dt, r.dh, 1)
        u = oracle.run(p, r.nt)
        l2, _ = oracle.errors(p, r.nt, u)
        assert l2 / (r.nx * r.ny) <= 1e-6


def test_tiled_equals_serial(oracle):
    # 2d_nonlocal_async execution model (tile tasks + barrier) == serial, bitwise
    for tiles in [(1, 1), (2, 2), (5, 3), (20, 20)]:
        p = oracle.params(40, 60, 5, 0.2, 0.001, 0.02, 1)
        ref = oracle.run(p, 7)
        u = oracle.test_init(p)
        oracle.run_tiled(p, 7, tiles[0], tiles[1], u, 4)
        assert np.array_equal(u, ref), tiles


def test_thread_count_invariance(oracle):
    p = oracle.params(37, 29, 4, 1.0, 0.0005, 0.02, 1)
    a = oracle.run(p, 5, nthreads=1)
    b = oracle.run(p, 5, nthreads=7)
    assert np.array_equal(a, b)


def test_disk_counts(oracle):
    # SURVEY.md 3.4 note 1
    for eps, n in [(3, 29), (5, 81), (6, 113), (8, 197), (10, 317), (16, 797), (32, 3209)]:
        assert oracle.disk_count(eps) == n
        assert N.disk_count(eps) == n


def test_golden_fields_reproduce(oracle):
    rows = {0: (50, 50, 45, 5, 1.0, 0.0005, 0.02), 5: (40, 40, 200, 3, 0.2, 0.001, 0.02),
            7: (40, 40, 200, 8, 0.2, 0.001, 0.02)}
    for r, (nx, ny, nt, eps, k, dt, dh) in rows.items():
        for test in (0, 1):
            g = np.load(os.path.join(GOLD, f"fields_2d_row{r}_test{test}.npy"))
            p = oracle.params(nx, ny, eps, k, dt, dh, test)
            assert np.array_equal(oracle.run(p, nt), g)


def test_per_step_l2_fixture(oracle):
    g = np.load(os.path.join(GOLD, "l2_per_step_row0.npy"))
    p = oracle.params(50, 50, 5, 1.0, 0.0005, 0.02, 1)
    u = oracle.test_init(p)
    for t in range(45):
        u = oracle.step(p, t, u)
        assert oracle.errors(p, t + 1, u)[0] == g[t]
    assert g[-1] == KA["serial_2d_txt"][0]["l2"]


def test_long_run_known_answer(oracle):
    a = KA["long_runs_eps8"][0]  # 64^2, eps=8, 1000 steps
    dh = 1.0 / a["nx"]
    dt = 8 ** 4 * dh * dh / (8 * 1.0 * oracle.disk_count(8))
    p = oracle.params(a["nx"], a["ny"], 8, 1.0, dt, dh, 1)
    u = oracle.run(p, a["nt"])
    l2, _ = oracle.errors(p, a["nt"], u)
    assert l2 == a["l2"]


def test_stdin_ic_order(oracle):
    # input_init reads sx outer (src/2d_nonlocal_serial.cpp:180-187): a stream
    # v0 v1 ... lands at index sx + sy*nx in sx-major order
    nx, ny = 3, 2
    stream = np.arange(nx * ny, dtype=np.float64)
    u = np.empty(nx * ny)
    i = 0
    for sx in range(nx):
        for sy in range(ny):
            u[sx + sy * nx] = stream[i]
            i += 1
    assert list(u) == [0, 2, 4, 1, 3, 5]


def test_linear_influence_restatement(oracle):
    """J(r) = 1 - r extension (problem_description.tex:149-159): c from M3 =
    1/20 (2/M3 = 40 in place of the reference's 8, pi omitted as :76), J = 1
    at the centre, 0 on the horizon; the J = 1 path is the pinned reference."""
    p1 = oracle.params(40, 30, 5, 1.0, 1e-4, 0.02, 0, 1)
    p0 = oracle.params(40, 30, 5, 1.0, 1e-4, 0.02, 0, 0)
    assert oracle.c2d(p1) == (1.0 * 40) / (5 * 0.02) ** 4
    assert oracle.c2d(p0) == (1.0 * 8) / (5 * 0.02) ** 4
    L = oracle.lib()
    import ctypes
    L.nlh_oracle_influence.argtypes = [ctypes.POINTER(type(p1)), ctypes.c_long, ctypes.c_long]
    L.nlh_oracle_influence.restype = ctypes.c_double
    assert L.nlh_oracle_influence(ctypes.byref(p1), 0, 0) == 1.0
    assert L.nlh_oracle_influence(ctypes.byref(p1), 3, 4) == 0.0
    assert L.nlh_oracle_influence(ctypes.byref(p0), 3, 4) == 1.0
    # a constant field is a fixed point of the operator away from the
    # boundary for any J (sum of J (u_j - u_i) = 0)
    u = np.ones((30, 40))
    un = oracle.step(p1, 0, u)
    assert np.allclose(un[10:20, 10:30], 1.0, rtol=0, atol=1e-15)


def test_oracle_1d_c_truncation(oracle):
    # `long c_1d` (src/1d_nonlocal_serial.cpp:57,74) truncates 3k/(eps dx)^3:
    # 2999.999... -> 2999 for the default flags, 0 for the last 1d.txt row
    assert oracle.lib().nlh_oracle_c1d(5, 1.0, 0.02) == 2999.0
    assert oracle.lib().nlh_oracle_c1d(40, 0.02, 0.016) == 0.0
    assert oracle.lib().nlh_oracle_c1d(40, 0.5, 0.02) == 2.0


def _parse_1d(text):
    tok = text.split()
    return [(int(tok[1 + 6 * i]), int(tok[2 + 6 * i]), int(tok[3 + 6 * i]), float(tok[4 + 6 * i]),
             float(tok[5 + 6 * i]), float(tok[6 + 6 * i])) for i in range(int(tok[0]))]


def test_oracle_1d_batch_contract(oracle):
    """Test_1d (CMakeLists.txt:101): every tests/1d.txt row has l2/nx <= 1e-6."""
    for nx, nt, eps, k, dt, dx in _parse_1d(read_input("1d.txt")):
        u = oracle.run_1d(nx, nt, eps, k, dt, dx, True)
        l2, li = oracle.errors_1d(nx, nt, dt, dx, u)
        assert l2 / nx <= 1e-6, (nx, nt, eps, l2)
        assert np.isfinite(u).all()


def test_oracle_1d_restatement_small(oracle):
    """The C restatement against a direct pure-Python transcription of
    sum_local / sum_local_test / do_work (1d :186-236) on a small case."""
    import math
    nx, nt, eps, k, dt, dx = 13, 7, 3, 1.0, 0.001, 0.02
    c = float(int((k * 3) / (pow(eps * dx, 3))))

    def w(pos, t):
        return math.cos(2 * math.pi * (t * dt)) * math.sin(2 * math.pi * (pos * dx))

    S = [[math.sin(2 * math.pi * (x * dx)) for x in range(nx)], [0.0] * nx]
    for t in range(nt):
        cur, nxt = S[t % 2], S[(t + 1) % 2]
        for x in range(nx):
            r = 0.0
            for sx in range(x - eps, x + eps + 1):
                r += 1.0 * c * ((cur[sx] if 0 <= sx < nx else 0.0) - cur[x]) * dx
            nxt[x] = cur[x] + (r * dt)
            r2 = -(2 * math.pi * math.sin(2 * math.pi * (t * dt)) * math.sin(2 * math.pi * (x * dx)))
            wp = w(x, t)
            for sx in range(x - eps, x + eps + 1):
                r2 -= 1.0 * c * ((w(sx, t) if 0 <= sx < nx else 0.0) - wp) * dx
            nxt[x] += r2 * dt
    u = oracle.run_1d(nx, nt, eps, k, dt, dx, True)
    assert u.tolist() == S[nt % 2]


def _direct_longdouble_step(oracle, p, u0):
    """One step by the disk loops themselves in numpy long double (x87 80-bit
    here and on the GPU box), rounded once: the compensated oracle's spec."""
    import math
    L = np.longdouble
    nx, ny, eps = p.nx, p.ny, p.eps
    c, dh2, dt = L(oracle.c2d(p)), L(p.dh * p.dh), L(p.dt)
    st, ct = L(math.sin(2 * math.pi * (0 * p.dt))), L(math.cos(2 * math.pi * (0 * p.dt)))
    sx = [L(math.sin(2 * math.pi * (i * p.dh))) for i in range(nx)]
    sy = [L(math.sin(2 * math.pi * (i * p.dh))) for i in range(ny)]
    n = oracle.disk_count(eps)
    out = np.zeros((ny, nx))
    for y in range(ny):
        for x in range(nx):
            su = sw = L(0)
            for dx in range(-eps, eps + 1):  # sx outer, as the reference
                ln = int(math.sqrt(eps * eps - dx * dx))
                for dy in range(-ln, ln + 1):
                    xx, yy = x + dx, y + dy
                    if 0 <= xx < nx and 0 <= yy < ny:
                        su += L(u0[yy, xx])
                        sw += ct * sx[xx] * sy[yy]
            ui = L(u0[y, x])
            r = c * dh2 * (su - n * ui)
            if p.test:
                w0 = sx[x] * sy[y]
                r += -(2 * L(math.pi) * st) * w0 - c * dh2 * (sw - n * (ct * w0))
            out[y, x] = float(ui + dt * r)
    return out


@pytest.mark.parametrize("test", [0, 1])
def test_compensated_oracle_is_the_longdouble_disk_sum(oracle, test):
    """oracle.run_compensated (row windows of long-double
    prefix sums) equals the disk loops evaluated in long double, rounded once
    -- bit for bit on a ragged lattice whose disk leaves the domain."""
    eps, nx, ny = 7, 23, 19
    dh = 1.0 / nx
    p = oracle.params(nx, ny, eps, 1.0, 0.3 * eps ** 4 * dh * dh / (8 * oracle.disk_count(eps)), dh, test)
    u0 = np.random.default_rng(1).uniform(-1, 1, (ny, nx))
    assert np.array_equal(oracle.run_compensated(p, 1, u0), _direct_longdouble_step(oracle, p, u0))


@pytest.mark.parametrize("eps,test", [(3, 1), (5, 1), (8, 0), (8, 1), (12, 1)])
def test_compensated_oracle_near_reference_order(oracle, eps, test):
    """Where the reference's N(eps) sequential terms round little (small eps),
    the compensated steps stay within a few ulp of field scale of the
    reference's own order over several steps at the stable dt (alpha N = 1)."""
    nx, ny = 50, 43
    dh = 1.0 / nx
    p = oracle.params(nx, ny, eps, 1.0, eps ** 4 * dh * dh / (8 * oracle.disk_count(eps)), dh, test)
    a, b = oracle.run(p, 5), oracle.run_compensated(p, 5)
    assert np.abs(a - b).max() <= 1e-14 * np.abs(a).max()
