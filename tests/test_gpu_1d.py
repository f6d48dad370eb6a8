"""GPU: the 1D solver (nlh1d_*, k_1d) against the oracle's restatement of
src/1d_nonlocal_serial.cpp, bit for bit, and the reference's Test_1d batch
contract (CMakeLists.txt:101, tests/1d.txt) through the Python mirror and the
bin/1d_nonlocal_serial drop-in.

Parity note: the reference ships no 1D outputs, so these cases are pinned by
the restatement (test_oracle.py::test_oracle_1d_restatement_small) and the
batch contract only.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import REF_TESTS, ROOT, read_input

import nonlocalheatequation_amd as N

pytestmark = pytest.mark.gpu


CASES = [  # nx nt eps k dt dx
    (50, 45, 5, 1.0, 0.001, 0.02),      # driver defaults (c = 2999)
    (1000, 50, 5, 1.0, 0.001, 0.02),
    (1000, 450, 40, 0.5, 0.001, 0.02),  # c = 2
    (100, 45, 40, 0.02, 0.005, 0.016),  # c = 0
    (7, 20, 9, 1.0, 0.001, 0.05),       # horizon wider than the lattice
    (1, 5, 3, 1.0, 0.001, 0.02),
    (70000, 6, 12, 1.0, 1e-6, 0.001),   # many workgroups
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("test", [True, False])
def test_1d_bitwise_vs_oracle(oracle, case, test):
    nx, nt, eps, k, dt, dx = case
    with N.Solver1D(nx, eps, k, dt, dx, test=test, device=0) as s:
        s.test_init()
        s.do_work(nt)
        got = s.field()
        want = oracle.run_1d(nx, nt, eps, k, dt, dx, test)
        assert np.array_equal(got, want)
        if test:
            l2, li = oracle.errors_1d(nx, nt, dt, dx, want)
            assert (s.error_l2, s.error_linf) == (l2, li)


def test_1d_input_init_and_split_runs(oracle):
    nx, eps, k, dt, dx = 333, 7, 1.0, 0.0005, 0.01
    u0 = np.random.default_rng(3).standard_normal(nx)
    with N.Solver1D(nx, eps, k, dt, dx, device=0) as s:
        s.input_init(u0)
        s.run(4)
        s.run(9)
        got = s.field()
    assert np.array_equal(got, oracle.run_1d(nx, 13, eps, k, dt, dx, False, u0))


def test_1d_batch_contract():
    assert N.batch_tester_1d(read_input("1d.txt")) == "Tests Passed"


def test_1d_bad_arguments():
    with pytest.raises(N.NLHError):
        N.Solver1D(0, 5, device=0)
    with pytest.raises(N.NLHError):
        N.Solver1D(10, 0, device=0)


def _run(args, stdin=None, cwd=None):
    p = subprocess.run([os.path.join(ROOT, "bin", "1d_nonlocal_serial"), *args], input=stdin,
                       capture_output=True, text=True, timeout=300, cwd=cwd)
    assert p.returncode == 0, p.stderr
    return p.stdout


def test_1d_driver_batch():
    out = _run(["--test_batch"], stdin=open(os.path.join(REF_TESTS, "1d.txt")).read())
    assert out.splitlines()[0].endswith("1d_nonlocal_serial (0.1.0)")
    assert "Tests Passed" in out


def test_1d_driver_test_mode(oracle):
    out = _run(["--test", "--results"]).splitlines()
    u = oracle.run_1d(50, 45, 5, 1.0, 0.001, 0.02, True)
    l2, li = oracle.errors_1d(50, 45, 0.001, 0.02, u)
    assert out[1] == f"l2: {l2:g} linfinity: {li:g}"
    exp = [l for l in out if l.startswith("Expected:")]
    res = [l for l in out if l.startswith("S[")]
    assert len(exp) == 50 and len(res) == 50
    assert [float(l.split("= ")[1]) for l in res] == pytest.approx(u.tolist(), rel=1e-5, abs=1e-12)
    # 1d timing line, no header (the reference's header flag starts false)
    assert not any(l.startswith("OS_Threads") for l in out)
    assert out[-1].split(",")[0].strip() == "1"


def test_1d_driver_stdin_and_logs(tmp_path, oracle):
    run_dir = tmp_path / "run"
    for d in ("run", "out_csv", "out_vtk"):
        (tmp_path / d).mkdir()
    u0 = np.linspace(-1, 1, 20)
    out = _run(["--nx", "20", "--nt", "11", "--eps", "3", "--results", "--nlog", "5"],
               stdin=" ".join(repr(float(v)) for v in u0), cwd=str(run_dir))
    want = oracle.run_1d(20, 11, 3, 1.0, 0.001, 0.02, False, u0)
    got = [float(l.split("= ")[1]) for l in out.splitlines() if l.startswith("S[")]
    assert got == pytest.approx(want.tolist(), rel=1e-5, abs=1e-12)
    rows = (tmp_path / "out_csv" / "simulate_1d.csv").read_text().splitlines()
    assert sorted({int(r.split(",")[0]) for r in rows}) == [0, 5, 10]
    assert sorted(os.listdir(tmp_path / "out_vtk")) == ["simulate_0.vtu", "simulate_1.vtu", "simulate_2.vtu"]
