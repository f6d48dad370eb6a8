"""GPU: the drop-in executables bin/2d_nonlocal_{serial,async,distributed}.

Mirrors the reference's CTest contract (CMakeLists.txt:101-154: run
`--test_batch < tests/<file>.txt`, pass on "Tests Passed") plus the stdout
formats, stdin IC order and the ../out_csv, ../out_vtk logging.
"""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import REF_TESTS, ROOT
from vtu import read_vtu

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "bin")


def run(exe, args=(), stdin=None, cwd=None, timeout=300):
    p = subprocess.run([os.path.join(BIN, exe), *args], input=stdin, capture_output=True, text=True,
                       cwd=cwd, timeout=timeout)
    assert p.returncode == 0, p.stderr
    return p.stdout


@pytest.mark.parametrize("exe,fname", [("2d_nonlocal_serial", "2d.txt"),
                                       ("2d_nonlocal_async", "2d_async.txt"),
                                       ("2d_nonlocal_distributed", "2d_distributed.txt")])
@pytest.mark.parametrize("kernel", ["auto", "fast"])
def test_batch_files_pass(exe, fname, kernel):
    out = run(exe, ["--test_batch", "--kernel", kernel], stdin=open(os.path.join(REF_TESTS, fname)).read())
    assert "Tests Passed" in out and "Tests Failed" not in out
    assert out.splitlines()[0].endswith(f"{exe} (0.1.0)")


def test_batch_failure_reported():
    # a stable but inaccurate row (l2/N > 1e-6) must print "Tests Failed"
    out = run("2d_nonlocal_serial", ["--test_batch"], stdin="1\n20 20 50 3 0.01 0.05 0.05\n")
    assert "Tests Failed" in out


def test_serial_test_mode_output(oracle):
    out = run("2d_nonlocal_serial", ["--test", "--cmp", "false", "--nlog", "1000"])
    lines = out.splitlines()
    p = oracle.params(50, 50, 5, 1.0, 0.0005, 0.02, 1)
    l2, li = oracle.errors(p, 45, oracle.run(p, 45))
    assert lines[1] == f"l2: {l2:g} linfinity: {li:g}"
    assert lines[2].startswith("OS_Threads,       Execution_Time_sec,")
    assert re.match(r"^1,\s+ [0-9.]+,\s+50,\s+50,\s+45 \s*$", lines[3]), lines[3]


def test_serial_cmp_and_results(oracle):
    out = run("2d_nonlocal_serial", ["--test", "--results", "--nx", "6", "--ny", "5", "--nt", "3",
                                     "--eps", "2", "--nlog", "1000", "--no-header"])
    lines = out.splitlines()
    exp = [l for l in lines if l.startswith("Expected:")]
    assert len(exp) == 30
    p = oracle.params(6, 5, 2, 1.0, 0.0005, 0.02, 1)
    u = oracle.run(p, 3)
    w = oracle.exact(p, 3)
    # sx outer, sy inner (src/2d_nonlocal_serial.cpp:119-123)
    assert exp[1] == f"Expected: {w[1, 0]:g} Actual: {u[1, 0]:g}"
    res = [l for l in lines if l.startswith("S[")]
    assert len(res) == 6 and res[0].startswith(f"S[0][0] = {u[0, 0]:g} S[0][1] = {u[1, 0]:g}")
    assert not any(l.startswith("OS_Threads") for l in lines)  # --no-header


def test_serial_stdin_ic(oracle):
    nx, ny, nt = 7, 5, 4
    rng = np.random.default_rng(3)
    u0 = rng.uniform(-1, 1, size=(ny, nx))
    stream = " ".join(repr(float(u0[sy, sx])) for sx in range(nx) for sy in range(ny))  # sx outer
    out = run("2d_nonlocal_serial", ["--results", "--nx", str(nx), "--ny", str(ny), "--nt", str(nt),
                                     "--eps", "2", "--nlog", "1000"], stdin=stream)
    vals = [float(v) for v in re.findall(r"S\[\d+\]\[\d+\] = (\S+)", out)]
    p = oracle.params(nx, ny, 2, 1.0, 0.0005, 0.02, 0)
    ref = oracle.run(p, nt, u0)
    got = np.array(vals).reshape(nx, ny).T
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-6)


def test_logging_csv_vtu(tmp_path, oracle):
    run_dir = tmp_path / "build"
    run_dir.mkdir()
    (tmp_path / "out_csv").mkdir()
    (tmp_path / "out_vtk").mkdir()
    run("2d_nonlocal_serial", ["--test", "--cmp", "false", "--nt", "11", "--nlog", "5", "--kernel", "exact"],
        cwd=run_dir)
    rows = open(tmp_path / "out_csv" / "simulate_2d.csv").read().splitlines()
    assert len(rows) == 3 * 2500  # t = 0, 5, 10
    assert rows[0].startswith("0,0,0,")
    score = open(tmp_path / "out_csv" / "score_2d.csv").read().splitlines()
    assert [s.split(",")[0] for s in score] == ["0", "5", "10"]
    p = oracle.params(50, 50, 5, 1.0, 0.0005, 0.02, 1)
    for idx, t in [(0, 0), (1, 5), (2, 10)]:
        npts, arr = read_vtu(tmp_path / "out_vtk" / f"simulate_{idx}.vtu")  # serial: t / nlog
        assert npts == 2500
        ref = oracle.run(p, t + 1)  # S[next] after step t
        assert np.array_equal(arr["Temperature"], ref.ravel())
        pts = arr["Points"].reshape(-1, 3)
        assert pts[51].tolist() == [1.0, 1.0, 0.0]


def test_async_vtk_named_by_step(tmp_path):
    run_dir = tmp_path / "b"
    run_dir.mkdir()
    (tmp_path / "out_vtk").mkdir()
    run("2d_nonlocal_async", ["--nt", "6", "--nlog", "5"], cwd=run_dir)
    assert sorted(os.listdir(tmp_path / "out_vtk")) == ["simulate_0.vtu", "simulate_5.vtu"]


def test_async_defaults_and_timing_line(oracle):
    out = run("2d_nonlocal_async", ["--no-header"])
    lines = out.splitlines()
    p = oracle.params(50, 50, 5, 1.0, 0.0005, 0.02, 1)  # 25x25 tiles x np=2
    l2, li = oracle.errors(p, 45, oracle.run(p, 45))
    assert lines[1] == f"l2: {l2:g} linfinity: {li:g}"
    assert re.match(r"^1,\s+ [0-9.]+,\s+25,\s+25,\s+45 \s*$", lines[2]), lines[2]


def test_distributed_file_and_format(oracle):
    f = os.path.join(REF_TESTS, "load_balance_4s_2n.txt")
    out = run("2d_nonlocal_distributed", ["--file", f, "--nt", "10", "--cmp", "true", "--nlog", "1000"])
    lines = out.splitlines()
    p = oracle.params(40, 40, 5, 1.0, 0.0005, 0.0025, 1)
    u = oracle.run(p, 10)
    l2, li = oracle.errors(p, 10, u)
    assert lines[1] == f"l2: {l2:g} linfinity: {li:g}"
    assert lines[2].startswith(f"sx: 0 sy: 0 Expected: ")
    hdr = [i for i, l in enumerate(lines) if l.startswith("Localities,OS_Threads")]
    assert hdr and re.match(r"^1,\s+1,\s+[0-9.e-]+, 20,\s+20,\s+2,\s+2,\s+10 \s*$", lines[hdr[0] + 1])


def test_distributed_small_tile_warning():
    out = run("2d_nonlocal_distributed", ["--nx", "4", "--ny", "4", "--eps", "5", "--nt", "2",
                                          "--dh", "0.05", "--nlog", "1000"])
    assert "[WARNING] Mesh size on a single node" in out


def test_hpx_flags_ignored():
    out = run("2d_nonlocal_serial", ["--hpx:threads=4", "--test", "--cmp", "false", "--nt", "2"])
    assert "l2:" in out


def test_serial_linear_influence_flag(oracle):
    """--influence linear (extra flag): J(r) = 1 - r with c from M3 = 1/20."""
    out = run("2d_nonlocal_serial", ["--test", "--cmp", "false", "--nt", "10", "--nlog", "1000",
                                     "--influence", "linear", "--kernel", "exact"])
    p = oracle.params(50, 50, 5, 1.0, 0.0005, 0.02, 1, 1)
    l2, li = oracle.errors(p, 10, oracle.run(p, 10))
    assert out.splitlines()[1] == f"l2: {l2:g} linfinity: {li:g}"
    p = subprocess.run([os.path.join(BIN, "2d_nonlocal_serial"), "--influence", "quadratic"],
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0



@pytest.mark.parametrize("eps", [70, 100])
def test_serial_driver_large_horizon(oracle, eps):
    """--eps past the compile-time horizons (the reference accepts any,
    src/2d_nonlocal_serial.cpp:403): the serial driver's AUTO route runs
    k_prefix_rt; its printed l2 / linfinity match the oracle's (6 digits)."""
    nx, nt = 160, 3
    dh = 1.0 / nx
    dt = 0.05 * eps ** 4 * dh * dh / (8 * oracle.disk_count(eps))
    out = run("2d_nonlocal_serial", ["--test", "--cmp", "false", "--nx", str(nx), "--ny", str(nx), "--nt", str(nt),
                                     "--eps", str(eps), "--dt", repr(dt), "--dh", repr(dh), "--nlog", "1000"])
    p = oracle.params(nx, nx, eps, 1.0, dt, dh, 1)
    l2, li = oracle.errors(p, nt, oracle.run(p, nt))
    m = re.search(r"^l2: (\S+) linfinity: (\S+)$", out, re.M)
    assert m and float(m.group(1)) == pytest.approx(l2, rel=1e-5) and float(m.group(2)) == pytest.approx(li, rel=1e-5)


def test_auto_kernel_choice_and_note(oracle):
    """--kernel auto in test mode runs EXACT where the whole
    run is cheap (nx*ny*nt*N(eps) <= 2e11 disk terms), so the printed l2 /
    linfinity are the reference's own order -- bit for bit with the oracle --
    and says nothing; past that it runs a FAST kernel and one stderr line
    names the kernel and the L2 contract."""
    p = subprocess.run([os.path.join(BIN, "2d_nonlocal_serial"), "--test", "--cmp", "false", "--nx", "120",
                        "--ny", "100", "--nt", "30", "--eps", "8", "--dh", repr(1 / 120), "--dt", "1e-6",
                        "--nlog", "1000"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "note:" not in p.stderr, p.stderr
    o = oracle.params(120, 100, 8, 1.0, 1e-6, 1 / 120, 1)
    l2, li = oracle.errors(o, 30, oracle.run(o, 30))
    assert p.stdout.splitlines()[1] == f"l2: {l2:g} linfinity: {li:g}"
    n = 1200  # 1200^2 * 800 * 197 = 2.3e11 terms: FAST
    p = subprocess.run([os.path.join(BIN, "2d_nonlocal_serial"), "--test", "--cmp", "false", "--nx", str(n),
                        "--ny", str(n), "--nt", "800", "--eps", "8", "--dh", repr(1 / n),
                        "--dt", repr(8 ** 4 / (n * n * 8 * 197)), "--nlog", "100000"],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    notes = [l for l in p.stderr.splitlines() if l.startswith("note: --kernel auto ran the FAST kernel")]
    assert len(notes) == 1 and "k_pair_split" in notes[0] and "--kernel exact" in notes[0], p.stderr
    assert p.stdout.splitlines()[1].startswith("l2: ")
