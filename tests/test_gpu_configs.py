"""GPU: BASELINE.json's multi-GPU configurations at full size on one MI355X,
and long-run parity.

* C3 (32768^2, eps=8, npx=2 x npy=4 blocks of 16384 x 8192): the eight
  blocks of the 8-GPU layout on one device, every halo piece packed, sent
  through ncclSend/ncclRecv (to self, NLH_RCCL_SELF) and unpacked -- the
  production two-step pass, checked per node against the bit-parity kernel
  k_exact on one block (bitwise equal to the reference's per-term order on
  every oracle-sized case), plus the bitwise linearity step(2u) = 2 step(u).
* C4 (8192^2, eps=32) in its 1x1, 2x2 and 2x4 layouts (RCCL to self): the
  large-horizon kernel k_wide vs k_exact per node, and linearity.
* C5 uneven (tests/load_balance_25s_8n.txt: 5 x 5 tiles of 9216^2 over 8
  owners, 1-7 tiles each, 2.1 G nodes = 16384^2 per GPU on average): the
  owners' blocks on one device (NLH_VIRTUAL_RANKS=8), pieces between owners
  over RCCL, checked against k_exact.
* Long runs: the fast kernels over 1000 steps against the reference's own
  known answers (long_runs_eps8: L2 of the reference
  serial solver at 64^2 and 96^2) and the two-step pass against the oracle.

Tolerances as tests/test_gpu_parity.py: 1e-12 of field scale per node, L2
within 1e-10 relative.
"""
import json
import os

import numpy as np
import pytest

from conftest import check_nodes, check_l2, ROOT, read_input, virtual_peer_pairs

import nonlocalheatequation_amd as N

pytestmark = pytest.mark.gpu

with open(os.path.join(ROOT, "tests", "golden", "known_answers.json")) as f:
    KNOWN = json.load(f)


def _dt(eps, dh, k=1.0):
    return eps ** 4 * dh * dh / (8 * k * N.disk_count(eps))


def _max_abs_diff(a, b, rows=2048):
    """max |a - b| and max |b| without full-size temporaries."""
    d = s = 0.0
    for y in range(0, a.shape[0], rows):
        x = a[y:y + rows]
        r = b[y:y + rows]
        d = max(d, float(np.max(np.abs(x - r))))
        s = max(s, float(np.max(np.abs(r))))
    return d, s


def _bitwise_double(a, b, rows=2048):
    for y in range(0, a.shape[0], rows):
        if not np.array_equal((2.0 * a[y:y + rows]).view(np.uint64), b[y:y + rows].view(np.uint64)):
            return False
    return True


def _run(nx, ny, eps, nt, kernel, u0=None, tiles=(1, 1), split=False, owner=None, test=False, ic_scale=None):
    dh = 1.0 / nx
    with N.Solver(nx, ny, eps, 1.0, _dt(eps, dh), dh, test=test, kernel=kernel, tiles=tiles,
                  split_tiles=split, owner=owner) as s:
        if u0 is None:
            s.test_init()
        else:
            s.input_init(u0)
        s.run(nt)
        s.synchronize()
        return s.field(), s.info()


@pytest.mark.parametrize("mode", ["rccl_self", "virtual8"])
def test_c3_blocks_over_rccl_self(monkeypatch, mode):
    """C3's 2 x 4 layout of 16384 x 8192 blocks (8.6 GB per field) through the
    RCCL transport, two two-step passes; vs k_exact per node, and linear.
    rccl_self: one rank, all eight blocks', every piece over RCCL to self;
    virtual8: eight virtual ranks with one block each, each with its own
    per-peer buffers (3-5 peers), every rank-to-rank message in one grouped
    exchange -- the 8-GPU run's message pattern."""
    n, eps, nt = 32768, 8, 4
    rng = np.random.default_rng(3)
    u0 = np.empty((n, n))
    for y in range(0, n, 4096):
        u0[y:y + 4096] = rng.uniform(-1.0, 1.0, size=(4096, n))
    env = ("NLH_RCCL_SELF", "1") if mode == "rccl_self" else ("NLH_VIRTUAL_RANKS", "8")
    monkeypatch.setenv(*env)
    uf, info = _run(n, n, eps, nt, "fast", u0, tiles=(2, 4), split=True)
    peers = 1 if mode == "rccl_self" else virtual_peer_pairs(n, n, eps, (2, 4), None, 8, split_tiles=True,
                                                             dt=_dt(eps, 1.0 / n), dh=1.0 / n)
    assert info.nblocks == 8 and info.npeers == peers and info.steps_per_pass == 2
    assert mode == "rccl_self" or peers == 32  # 2x4 blocks: 4 corner ranks x 3 peers + 4 inner x 5
    assert info.halo_width == 2 * eps and info.halo_bytes_sent > 0
    monkeypatch.delenv(env[0])
    ue, info_e = _run(n, n, eps, nt, "exact", u0)
    assert info_e.kernel == N.KERNEL_EXACT and info_e.nblocks == 1
    check_nodes(uf, ue, "C3 / C4 / C5 layout vs k_exact")
    del ue
    # linearity of the explicit step (test=0): every add, multiply and fma of
    # the pass commutes with scaling by 2, so step(2u) == 2 step(u) bitwise
    u0 *= 2.0
    monkeypatch.setenv(*env)
    u2, _ = _run(n, n, eps, nt, "fast", u0, tiles=(2, 4), split=True)
    assert _bitwise_double(uf, u2)


def test_c3_full_run_length_virtual8(monkeypatch):
    """C3 at its stated run length (200 steps; src/2d_nonlocal_distributed.cpp's
    strong-scaling run, BASELINE.json configs[2]): the 2 x 4 blocks of
    16384 x 8192 as eight virtual ranks -- every halo strip over grouped RCCL
    send/recv, 100 two-step passes -- against 200 steps of k_exact on one
    block (~20 s), per node (check_nodes, chunked: no full-size temporaries)."""
    n, eps, nt = 32768, 8, 200
    rng = np.random.default_rng(5)
    u0 = np.empty((n, n))
    for y in range(0, n, 4096):
        u0[y:y + 4096] = rng.uniform(-1.0, 1.0, size=(4096, n))
    monkeypatch.setenv("NLH_VIRTUAL_RANKS", "8")
    uf, info = _run(n, n, eps, nt, "fast", u0, tiles=(2, 4), split=True)
    assert info.nblocks == 8 and info.steps_per_pass == 2 and info.halo_bytes_sent > 0
    monkeypatch.delenv("NLH_VIRTUAL_RANKS")
    ue, info_e = _run(n, n, eps, nt, "exact", u0)
    assert info_e.kernel == N.KERNEL_EXACT and info_e.nblocks == 1
    del u0
    check_nodes(uf, ue, "C3 200 steps, 2x4 virtual ranks vs one-block k_exact")


@pytest.mark.parametrize("test", [False, True])
def test_c4_run_length_wide_vs_exact(test):
    """C4 at its run length: 100 steps (BASELINE C4: nt = 100) at 8192^2,
    eps = 32, k_wide vs the bit-parity k_exact per node, 1e-12 of field
    scale -- rounding drift of the prefix-sum windows over a whole run, in
    production and test mode (test_init IC; L2 within 1e-10 relative)."""
    n, eps, nt = 8192, 32, 100
    dh = 1.0 / n
    res = {}
    for kernel in ("fast", "exact"):
        with N.Solver(n, n, eps, 1.0, _dt(eps, dh), dh, test=test, kernel=kernel) as s:
            s.test_init()
            s.run(nt)
            s.synchronize()
            res[kernel] = (s.field(), s.errors(nt) if test else None, s.info())
    uf, ef, info = res["fast"]
    ue, ee, info_e = res["exact"]
    assert info.pass_kernel == "k_wide" and info_e.kernel == N.KERNEL_EXACT
    check_nodes(uf, ue, "C3 / C4 / C5 layout vs k_exact")
    if test:
        # 1e-10 relative (or of the rounding floor), recorded
        check_l2(ef[0], ee[0], uf, ue, "C4 100 steps k_wide vs k_exact")


@pytest.mark.parametrize("tiles", [(1, 1), (2, 2), (2, 4)])
def test_c4_full_size_wide_kernel(monkeypatch, tiles):
    """C4 (8192^2, eps=32, N=3209) at full size in its 1-, 4- and 8-GPU block
    layouts (blocks exchanging eps-wide halos over RCCL to self): k_wide with
    prefix-sum row windows, two steps, per node vs k_exact (the reference's
    per-term order), plus the bitwise linearity step(2u) = 2 step(u)."""
    n, eps, nt = 8192, 32, 2
    rng = np.random.default_rng(32)
    u0 = rng.uniform(-1.0, 1.0, size=(n, n))
    split = tiles != (1, 1)
    if split:
        monkeypatch.setenv("NLH_RCCL_SELF", "1")
    uf, info = _run(n, n, eps, nt, "fast", u0, tiles=tiles, split=split)
    assert info.pass_kernel == "k_wide" and info.nblocks == tiles[0] * tiles[1]
    monkeypatch.delenv("NLH_RCCL_SELF", raising=False)
    ue, info_e = _run(n, n, eps, nt, "exact", u0)
    assert info_e.kernel == N.KERNEL_EXACT
    check_nodes(uf, ue, "C3 / C4 / C5 layout vs k_exact")
    del ue
    if split:
        monkeypatch.setenv("NLH_RCCL_SELF", "1")
    u2, _ = _run(n, n, eps, nt, "fast", 2.0 * u0, tiles=tiles, split=split)
    assert _bitwise_double(uf, u2)


def test_c5_uneven_owner_map_virtual_ranks(monkeypatch):
    """C5's uneven case: tests/load_balance_25s_8n.txt over 5 x 5 tiles of
    9216^2 (46080^2, 17 GB per field); each of the 8 owners' tiles merged into
    its own blocks, pieces between owners over RCCL (to self).  One two-step
    pass plus one single step (odd nt) from the test_init IC, vs k_exact."""
    tok = read_input("load_balance_25s_8n.txt").split()
    npx, npy = int(tok[2]), int(tok[3])
    owner = [0] * (npx * npy)
    vals = list(map(int, tok[5:]))
    for i in range(npx * npy):
        px, py, loc = vals[3 * i:3 * i + 3]
        owner[px + py * npx] = loc
    tile, eps, nt = 9216, 8, 3
    n = tile * npx
    monkeypatch.setenv("NLH_VIRTUAL_RANKS", "8")
    uf, info = _run(n, n, eps, nt, "fast", None, tiles=(npx, npy), owner=owner)
    plan = N.block_plan(n, n, eps, (npx, npy), owner, 8, False)
    pairs = virtual_peer_pairs(n, n, eps, (npx, npy), owner, 8, dt=_dt(eps, 1.0 / n), dh=1.0 / n)
    assert info.nblocks == len(plan) > 8 and info.npeers == pairs > 8 and info.halo_bytes_sent > 0
    assert info.steps_per_pass == 2
    monkeypatch.delenv("NLH_VIRTUAL_RANKS")
    ue, _ = _run(n, n, eps, nt, "exact", None)
    check_nodes(uf, ue, "C3 / C4 / C5 layout vs k_exact")


@pytest.mark.parametrize("kernel", ["fast", "auto", "exact"])
@pytest.mark.parametrize("case", range(len(KNOWN["long_runs_eps8"])))
def test_long_run_l2_known_answers(kernel, case):
    """1000 test-mode steps at eps=8 (64^2, 96^2): the L2 error of the
    reference serial solver itself within 1e-10
    relative -- the fast kernels' reordered sums must not drift."""
    ka = KNOWN["long_runs_eps8"][case]
    nx, ny, nt, eps = ka["nx"], ka["ny"], ka["nt"], ka["eps"]
    dh = 1.0 / nx
    with N.Solver(nx, ny, eps, 1.0, _dt(eps, dh), dh, test=True, kernel=kernel) as s:
        s.test_init()
        s.do_work(nt)
        info = s.info()
        l2 = s.error_l2
    assert info.kernel == (N.KERNEL_EXACT if kernel == "exact" else N.KERNEL_FAST)
    tol = 1e-13 if kernel == "exact" else 1e-10
    assert abs(l2 - ka["l2"]) <= tol * ka["l2"], f"l2 {l2!r} vs {ka['l2']!r}: rel {abs(l2 - ka['l2']) / ka['l2']:.3e}"


def test_long_run_two_step_pass_vs_oracle(oracle):
    """1000 production steps (500 two-step passes) at 256^2, eps=8, random IC,
    vs the oracle per node."""
    nx = ny = 256
    eps, nt = 8, 1000
    dh = 1.0 / nx
    dt = _dt(eps, dh)
    u0 = np.random.default_rng(1000).uniform(-1.0, 1.0, size=(ny, nx))
    u, info = _run(nx, ny, eps, nt, "fast", u0)
    assert info.steps_per_pass == 2
    ref = oracle.run(oracle.params(nx, ny, eps, 1.0, dt, dh, 0), nt, u0)
    scale = np.max(np.abs(ref))
    check_nodes(u, ref, scale=scale)


def test_bench_line_uneven_tile_map():
    """bench.py --map: the reference's uneven map (load_balance_25s_8n) as 8
    virtual owners on this GPU, small tiles -- the line names the map, the
    owners' tile counts and carries the exchange report."""
    import subprocess
    import sys
    m = os.path.join(ROOT, "tests", "golden", "reference_inputs", "load_balance_25s_8n.txt")
    env = dict(os.environ, NLH_VIRTUAL_RANKS="8")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--map", m, "--tile", "512",
                          "--steps", "4", "--warmup", "2", "--warmup-ms", "0", "--pmc", "off",
                          "--no-cpu-baseline", "--phase-passes", "4"],
                         capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads(out.stdout.strip().splitlines()[-1])
    c = line["config"]
    assert c["lattice"] == [2560, 2560] and c["tile_map"] == "load_balance_25s_8n.txt"
    assert c["virtual_ranks"] == 8 and sum(c["tiles_per_owner"]) == 25 and min(c["tiles_per_owner"]) >= 1
    assert line["value"] > 0 and line["scaling"] == "strong" and line["exchange"]["passes_timed"] > 0
