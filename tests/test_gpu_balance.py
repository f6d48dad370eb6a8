"""GPU: dynamic load balancing (nlh_repartition / nlh_rebalance; the
reference's load_balance, src/2d_nonlocal_distributed.cpp:844-959,
1306-1309) on one MI355X.

NLH_VIRTUAL_RANKS=V runs V owners' blocks on this GPU with the inter-owner
pieces over RCCL (to self), so a repartition exercises the multi-rank tile
move logic (RCCL refuses two real ranks on one device).  The field must be
carried across the repartition untouched: the run continues bit for bit as
the oracle (exact kernel) or within 1e-12 of field scale (fast kernels).
"""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import check_nodes, ROOT, read_input

import nonlocalheatequation_amd as N

pytestmark = pytest.mark.gpu


def _map(name):
    tok = read_input(name).split()
    npx, npy = int(tok[2]), int(tok[3])
    own = np.zeros(npx * npy, np.int32)
    vals = list(map(int, tok[5:]))
    for i in range(npx * npy):
        px, py, loc = vals[3 * i:3 * i + 3]
        own[px + py * npx] = loc
    return npx, npy, own, int(own.max()) + 1


def _check(oracle, u, p, t, kernel, u0=None):
    ref = oracle.run(p, t, u0)
    if kernel == "exact":
        assert np.array_equal(u, ref)
    else:
        check_nodes(u, ref)


@pytest.mark.parametrize("kernel,test,n1,n2", [("exact", True, 4, 3), ("fast", True, 3, 4),
                                               ("auto", False, 5, 6)])
def test_rebalance_virtual_ranks(oracle, monkeypatch, kernel, test, n1, n2):
    monkeypatch.setenv("NLH_VIRTUAL_RANKS", "4")
    npx, npy, own, R = _map("load_balance_25s_4n.txt")
    nx = ny = 5 * 48
    eps = 6
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    p = oracle.params(nx, ny, eps, 1.0, dt, dh, int(test))
    with N.Solver(nx, ny, eps, 1.0, dt, dh, test=test, kernel=kernel, tiles=(npx, npy), owner=own,
                  split_tiles=False) as s:
        s.test_init()
        s.kernel_timing(2)
        s.run(n1)
        s.synchronize()
        # each virtual rank's own measured stencil time (its launches timed
        # separately); at this size launch overhead dominates them, so the
        # rounds below are driven by busy = owned tiles (one unit per tile)
        m0, _, busy = s.rebalance(apply=False)
        assert m0 == 0 and busy.shape == (R,) and (busy > 0).all()
        cur = own.copy()
        moved, new, busy = s.rebalance(busy=np.bincount(cur, minlength=R).astype(float))
        assert moved > 0
        assert s.step_index == n1
        _check(oracle, s.field(), p, n1, kernel)
        t = n1
        for _ in range(4):  # rounds as every nbalance steps, until the map settles
            s.run(1)
            t += 1
            m, new, busy = s.rebalance(busy=np.bincount(new, minlength=R).astype(float))
            if m == 0:
                break
        cnt = np.bincount(new, minlength=R)
        assert m == 0 and cnt.max() - cnt.min() <= 1
        s.run(n2)
        s.synchronize()
        t += n2
        _check(oracle, s.field(), p, t, kernel)
        if test:
            l2, li = s.errors(t)
            rl2, rli = oracle.errors(p, t, oracle.run(p, t))
            assert l2 == pytest.approx(rl2, rel=1e-9) and li == pytest.approx(rli, rel=1e-9)


@pytest.mark.parametrize("kernel,test", [("exact", False), ("exact", True), ("fast", True), ("auto", False)])
def test_repartition_explicit_maps(oracle, monkeypatch, kernel, test):
    """Random maps over 3 virtual ranks: tiles move in every direction between
    every rank pair, each (sender, receiver) message through RCCL (to self)
    in tile order, then the run continues -- bitwise vs the oracle (exact) or
    within 1e-12 of field scale (fast), in production and test mode."""
    monkeypatch.setenv("NLH_VIRTUAL_RANKS", "3")
    nx, ny, eps, tiles = 180, 120, 5, (6, 4)
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    rng = np.random.default_rng(3)
    u0 = None if test else rng.uniform(-1, 1, size=(ny, nx))
    p = oracle.params(nx, ny, eps, 1.0, dt, dh, int(test))
    maps = [rng.integers(0, 3, 24).astype(np.int32) for _ in range(3)]
    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel=kernel, test=test, tiles=tiles, owner=maps[0]) as s:
        if test:
            s.test_init()
        else:
            s.input_init(u0)
        t = 0
        for m, n in zip(maps[1:] + [maps[1]], (2, 3, 1)):
            s.run(n)
            t += n
            s.repartition(m)
            assert s.step_index == t
        s.run(2)
        s.synchronize()
        _check(oracle, s.field(), p, t + 2, kernel, u0)
        with pytest.raises(N.NLHError):
            s.repartition(np.full(24, 3, np.int32))  # owner outside [0, 3)


def test_virtual_busy_measured_per_rank(monkeypatch):
    """Busy time under NLH_VIRTUAL_RANKS is each virtual rank's own measured
    stencil time: busy timing runs every rank's launch groups one after
    another on one stream (no other rank's kernels beside them), each launch
    group sized for the whole GPU as on the rank's own GPU, with the measured
    empty-launch overhead subtracted.  On an uneven map (1, 5, 4, 6 tiles of
    8192^2) busy time per tile agrees across ranks within 1.6x, so the busy
    times follow the work; rebalancing from them evens the measured busy
    times (spread <= 1.5x); the field after the moves matches
    the same run on one block (fast kernel: 1e-12 of field scale)."""
    monkeypatch.setenv("NLH_VIRTUAL_RANKS", "4")
    T = 4
    own = np.array([0, 1, 1, 1,
                    1, 1, 2, 2,
                    2, 2, 3, 3,
                    3, 3, 3, 3], np.int32)  # 1, 5, 4, 6 tiles
    # 8192^2 tiles: at 4096^2 the band launches and per-launch tails of the
    # small ranks put the per-tile spread at 1.7x (busy [2.17, 7.89, 8.00,
    # 7.66] ms, profiles/r04/first/pytest_gpu.log)
    nx = ny = T * 8192
    eps = 8
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="fast", tiles=(T, T), owner=own) as s:
        s.test_init()
        s.run(4)  # warm-up
        s.kernel_timing(2)
        s.run(40)
        s.synchronize()
        _, _, busy0 = s.rebalance(apply=False)
        per_tile = busy0 / np.bincount(own, minlength=4)
        assert (busy0 > 0).all() and per_tile.max() <= 1.6 * per_tile.min(), (busy0, per_tile)
        cur = own
        seen = []  # (measured spread, map it was measured on)
        for _ in range(8):
            s.kernel_timing(2)
            s.run(20)
            prev = cur
            m, cur, busy = s.rebalance()
            seen.append((float(busy.max() / busy.min()), prev.tolist()))
            if m == 0:
                break
        s.kernel_timing(2)
        s.run(20)
        s.synchronize()
        _, _, busy1 = s.rebalance(apply=False)
        seen.append((float(busy1.max() / busy1.min()), cur.tolist()))
        # the policy evens measured TIME, not tile counts: blocks of different
        # shapes run at different rates (r04: 3 / 5 / 4 / 4 tiles balanced).
        # Per-tile time depends on the block shape a rank's tiles form (r06: a
        # 1 x 4 column of tiles, left / right edge bands along its whole length,
        # 3.46 ms per tile against 2.5 for the others), so the tile moves can
        # cycle between maps near the optimum instead of stopping at one: the
        # assertion is on the maps the rounds measured -- one of them within
        # 1.5x and well below the start -- not on wherever round 8 left it
        # (round 6: final spreads 1.72 / 1.76 in two of three runs, each after
        # balanced maps earlier in the sequence)
        spread0 = busy0.max() / busy0.min()
        best = min(sp for sp, _ in seen)
        assert best <= 1.5 and best < 0.5 * spread0 and seen[-1][0] < 0.5 * spread0, (busy0, busy1, seen)
        s.run(6)
        s.synchronize()
        u = s.field()
        t = s.step_index
    monkeypatch.delenv("NLH_VIRTUAL_RANKS")
    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="fast") as r:
        r.test_init()
        r.run(t)
        ref = r.field()
    check_nodes(u, ref)


@pytest.mark.parametrize("target", [
    [0, 0, 1, 1, 0, 0, 1, 1, 2, 2, 3, 3, 2, 2, 3, 3],   # 3 tiles 1 -> 0, 2 -> 1, 3 -> 2
    [0, 1, 1, 1, 0, 1, 2, 2, 2, 2, 3, 3, 0, 3, 3, 3],   # 1 -> 0 and 3 -> 0 into two new blocks
])
def test_repartition_large_messages(monkeypatch, target):
    """Tile moves at 8192^2 tiles: the 1 / 5 / 4 / 6 map -> an even one sends
    three tiles (1.5 GiB) from rank 1 to rank 0 in one message into a freshly
    allocated 2 x 2-tile block; the other map moves two tiles into two new
    blocks of rank 0; the root gather of rank 3's six tiles is 3 GiB.  The
    gathered field, and the field after the move stepped on, match one block
    (fast kernel: 1e-12 of field scale).  Two round-4 fixes are under test
    (profiles/r04/{fourth,fifth,sixth}/diag_8192.log): messages go as
    <= 256 MiB chunks (unchunked, the 1.5 GiB message delivered only its first
    tile and the 3 GiB gather arrived corrupted), and a new solver zeroes its
    blocks on its own stream and waits (a null-stream memset could land after
    the moved tiles and zero them)."""
    monkeypatch.setenv("NLH_VIRTUAL_RANKS", "4")
    T = 4
    own = np.array([0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 3, 3], np.int32)
    nx = ny = T * 8192
    eps = 8
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="fast", tiles=(T, T), owner=own) as s:
        s.test_init()
        s.run(4)
        g = s.gather(0)
        s.repartition(np.array(target, np.int32))
        s.run(6)
        s.synchronize()
        u = s.field()
    monkeypatch.delenv("NLH_VIRTUAL_RANKS")
    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="fast") as r:
        r.test_init()
        r.run(4)
        ref4 = r.field()
        r.run(6)
        ref = r.field()
    scale = np.max(np.abs(ref))
    check_nodes(g, ref4, scale=scale)
    del g, ref4
    check_nodes(u, ref, scale=scale)


def test_busy_time_within_wall_time():
    """Busy timing serialises a pass's kernels on one stream, so a rank's busy
    time never exceeds the wall time of the window (the reference's busy rate
    10000 - idle-rate lies in [0, 10000]) -- here one rank with 2 x 2 blocks
    whose bands and interiors would otherwise overlap on two streams."""
    import time
    nx = ny = 8192
    eps = 8
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="fast", tiles=(2, 2), split_tiles=True) as s:
        s.test_init()
        s.run(4)
        s.synchronize()
        s.kernel_timing(2)
        t0 = time.perf_counter()
        s.run(100)
        s.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3
        busy_ms, steps = s.kernel_time()
    assert steps == 100 and 0 < busy_ms <= wall_ms, (busy_ms, wall_ms)
    assert busy_ms > 0.5 * wall_ms  # the GPU is busy most of the window


def test_phase_timing_reports_exchange(monkeypatch):
    """Phase timing (nlh_kernel_timing 3) on 2 x 2 blocks over RCCL to self:
    interior, band and exchange times per pass, wall >= interior, and the
    field equals an untimed run's bitwise (timing changes no arithmetic)."""
    monkeypatch.setenv("NLH_RCCL_SELF", "1")
    nx = ny = 4096
    eps = 8
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    out = {}
    for timed in (False, True):
        with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="fast", tiles=(2, 2), split_tiles=True) as s:
            s.test_init()
            if timed:
                s.kernel_timing(3)
            s.run(40)
            s.synchronize()
            out[timed] = s.field()
            if timed:
                ph = s.phase_time()
                assert ph.passes == 20 and ph.steps == 40
                assert ph.interior_ms > 0 and ph.band_ms > 0 and ph.exchange_ms > 0
                assert ph.wall_ms >= ph.interior_ms and ph.exposed_exchange_ms >= 0
                ms, steps = s.kernel_time()
                assert steps == 40 and ms == pytest.approx(ph.wall_ms)
    assert np.array_equal(out[False].view(np.uint64), out[True].view(np.uint64))


def test_rebalance_one_rank_measured():
    nx = ny = 256
    eps = 4
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    with N.Solver(nx, ny, eps, 1.0, dt, dh, tiles=(2, 2)) as s:
        s.test_init()
        with pytest.raises(N.NLHError):
            s.rebalance()  # busy timing is off
        s.kernel_timing(2)
        s.run(6)
        ms, steps = s.kernel_time()
        assert ms > 0 and steps == 6
        moved, own, busy = s.rebalance()
        assert moved == 0 and list(own) == [0, 0, 0, 0] and busy[0] == pytest.approx(ms)


def _scaled_map(tmp_path, name, tile):
    npx, npy, own, R = _map(name)
    lines = [f"{tile} {tile} {npx} {npy} {1.0 / (tile * npx)}"]
    lines += [f"{px} {py} {own[px + py * npx]}" for px in range(npx) for py in range(npy)]
    f = tmp_path / "map.txt"
    f.write_text("\n".join(lines) + "\n")
    return f, npx, npy, own, R


def test_driver_nbalance_virtual_ranks(oracle, tmp_path):
    """2d_nonlocal_distributed --nbalance over the reference's 25-tile map
    load_balance_25s_4n (21 of 25 tiles on one locality) on 4 virtual owners,
    small tiles: the report's format and the field through 4 repartitions
    (l2 as the oracle's).  The balancing verdict is checked at a tile size
    where busy time follows work (test_driver_balances_large_tiles)."""
    f, npx, npy, own, R = _scaled_map(tmp_path, "load_balance_25s_4n.txt", 32)
    env = dict(os.environ, NLH_VIRTUAL_RANKS=str(R))
    nt, dt = 45, 3e-5  # stable for eps 5 at dh = 1/160
    out = subprocess.run([os.path.join(ROOT, "bin", "2d_nonlocal_distributed"), "--file", str(f),
                          "--nt", str(nt), "--dt", str(dt), "--eps", "5", "--nbalance", "10",
                          "--test_load_balance", "--nlog", "1000"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    i = lines.index("Testing load balance:")
    rates = [float(l.split(": ")[-1]) for l in lines if l.startswith("Test: counter value: ")]
    assert len(rates) == R and all(0 <= r <= 10000 for r in rates) and sum(rates) <= 10000 * 1.001, rates
    assert any(l.startswith("Expected busy rate ") for l in lines)
    j = lines.index("Visualizing Load Balance across nodes")
    grid = [list(map(int, lines[j + 1 + r].split())) for r in range(npx)]
    cnt = np.bincount(np.array(grid).ravel(), minlength=R)
    assert cnt.sum() == npx * npy and cnt.min() >= 1 and i < j
    assert lines[j + 1 + npx] in ("Load balanced correctly", "Load not balanced correctly")
    # the field went through 4 repartitions untouched: l2 as the oracle's
    n = 32 * npx
    p = oracle.params(n, n, 5, 1.0, dt, 1.0 / n, 1)
    l2, li = oracle.errors(p, nt, oracle.run(p, nt))
    m = re.search(r"^l2: (\S+) linfinity: (\S+)$", out.stdout, re.M)
    assert m and float(m.group(1)) == pytest.approx(l2, rel=1e-5) and float(m.group(2)) == pytest.approx(li, rel=1e-5)


@pytest.mark.parametrize("nbal", [1, 3, 10])
def test_driver_nbalance_busy_window(oracle, tmp_path, nbal):
    """--nbalance WITHOUT --test_load_balance: busy timing runs only
    in a window of at most nbalance steps before each balance point (the rest
    of each interval keeps the overlapped exchange schedule).  --nbalance 1
    used to leave the window closed after the first balance and die in the
    second nlh_rebalance ('busy timing is off'); every interval length must
    run through, and the field through the repartitions stays the oracle's."""
    f, npx, npy, own, R = _scaled_map(tmp_path, "load_balance_25s_4n.txt", 32)
    env = dict(os.environ, NLH_VIRTUAL_RANKS=str(R))
    nt, dt = 12, 3e-5
    out = subprocess.run([os.path.join(ROOT, "bin", "2d_nonlocal_distributed"), "--file", str(f),
                          "--nt", str(nt), "--dt", str(dt), "--eps", "5", "--nbalance", str(nbal),
                          "--nlog", "1000"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr
    n = 32 * npx
    p = oracle.params(n, n, 5, 1.0, dt, 1.0 / n, 1)
    l2, li = oracle.errors(p, nt, oracle.run(p, nt))
    m = re.search(r"^l2: (\S+) linfinity: (\S+)$", out.stdout, re.M)
    assert m and float(m.group(1)) == pytest.approx(l2, rel=1e-5) and float(m.group(2)) == pytest.approx(li, rel=1e-5)


def test_driver_balances_large_tiles(tmp_path):
    """The same map with 2048^2 tiles (10240^2 lattice): busy time is kernel
    work, so after the --nbalance rounds the reference's verdict (:682-685:
    every busy rate within 1500 of the mean) reads "Load balanced correctly"
    -- the map evens measured time, so tile counts may differ by more than
    one (r04: 6 / 5 / 7 / 7 tiles at rates 2025 / 1823 / 2410 / 2148) -- the
    rates are within [0, 10000] and sum to at most 10000 (the owners share
    one GPU), and the run still passes the batch contract l2/N <= 1e-6."""
    f, npx, npy, own, R = _scaled_map(tmp_path, "load_balance_25s_4n.txt", 2048)
    env = dict(os.environ, NLH_VIRTUAL_RANKS=str(R))
    n = 2048 * npx
    eps, nt, nbal = 5, 60, 10
    dh = 1.0 / n
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    out = subprocess.run([os.path.join(ROOT, "bin", "2d_nonlocal_distributed"), "--file", str(f),
                          "--nt", str(nt), "--dt", repr(dt), "--eps", str(eps), "--nbalance", str(nbal),
                          "--test_load_balance", "--nlog", "100000"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    rates = [float(l.split(": ")[-1]) for l in lines if l.startswith("Test: counter value: ")]
    j = lines.index("Visualizing Load Balance across nodes")
    grid = [list(map(int, lines[j + 1 + r].split())) for r in range(npx)]
    cnt = np.bincount(np.array(grid).ravel(), minlength=R)
    assert cnt.min() >= 1 and all(0 <= r <= 10000 for r in rates) and sum(rates) <= 10000 * 1.001, (rates, cnt)
    assert lines[j + 1 + npx] == "Load balanced correctly", (rates, cnt)
    # the reference's verdict (|rate - mean| <= 1500) is loose once the four
    # owners share one GPU (rates ~2000-2500): the spread itself
    # must be small -- max / min <= 1.5 (r04: 2410 / 1823 = 1.32)
    assert max(rates) <= 1.5 * min(rates), (rates, cnt)
    m = re.search(r"^l2: (\S+) linfinity: (\S+)$", out.stdout, re.M)
    assert m and float(m.group(1)) / (n * n) <= 1e-6


def test_driver_runs_partitioner_file(oracle, tmp_path):
    """bin/2d_domain_decomposition (RCB partitioner) -> --file -> the
    distributed driver over 4 virtual owners: same L2 as the oracle."""
    f = tmp_path / "rcb.txt"
    p = subprocess.run([os.path.join(ROOT, "bin", "2d_domain_decomposition"), "160x160:0.00625", str(f), "4"],
                       input="32\n32\n", capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    env = dict(os.environ, NLH_VIRTUAL_RANKS="4")
    nt, dt = 20, 3e-5
    out = subprocess.run([os.path.join(ROOT, "bin", "2d_nonlocal_distributed"), "--file", str(f), "--nt", str(nt),
                          "--dt", str(dt), "--eps", "5", "--nlog", "1000"],
                         capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr
    pp = oracle.params(160, 160, 5, 1.0, dt, 0.00625, 1)
    l2, li = oracle.errors(pp, nt, oracle.run(pp, nt))
    m = re.search(r"^l2: (\S+) linfinity: (\S+)$", out.stdout, re.M)
    assert m and float(m.group(1)) == pytest.approx(l2, rel=1e-5) and float(m.group(2)) == pytest.approx(li, rel=1e-5)


def test_repartition_without_memory_leaves_solver_unchanged(oracle, monkeypatch):
    """A repartition needs the new solver beside the old one: with too little
    free device memory nlh_repartition fails with NLH_ERR_NOMEM (status 6)
    before allocating or sending anything, the field and step index stay as
    they were, and the run continues (bitwise vs the oracle, exact kernel);
    with the memory back the same repartition goes through."""
    import ctypes
    monkeypatch.setenv("NLH_VIRTUAL_RANKS", "2")
    N.lib()
    # the HIP runtime libnlh runs on (the copy already mapped in this process:
    # loading a second one by path would clash with the loaded HSA runtime)
    with open("/proc/self/maps") as f:
        paths = sorted({ln.split()[-1] for ln in f if "libamdhip64.so" in ln})
    assert paths, "no HIP runtime mapped"
    hip = ctypes.CDLL(paths[0])
    nx, ny, eps, tiles = 2048, 2048, 4, (4, 4)
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    p = oracle.params(nx, ny, eps, 1.0, dt, dh, 1)
    own0 = np.repeat(np.arange(2, dtype=np.int32), 8)
    own1 = own0[::-1].copy()
    held = []

    def free_bytes():
        f, t = ctypes.c_size_t(), ctypes.c_size_t()
        assert hip.hipMemGetInfo(ctypes.byref(f), ctypes.byref(t)) == 0
        return f.value

    with N.Solver(nx, ny, eps, 1.0, dt, dh, kernel="exact", test=True, tiles=tiles, owner=own0) as s:
        s.test_init()
        s.run(2)
        s.synchronize()
        before = s.field()
        try:
            target = 96 << 20  # leave less than the new solver needs (~2 x 35 MB + 64 MiB margin)
            chunk = 16 << 30
            while free_bytes() > target + (8 << 20) and chunk >= (1 << 20):
                ptr = ctypes.c_void_p()
                size = min(chunk, free_bytes() - target)
                if hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(size)) == 0:
                    held.append(ptr)
                else:
                    chunk //= 2
            with pytest.raises(N.NLHError, match=r"status 6"):
                s.repartition(own1)
        finally:
            for ptr in held:
                hip.hipFree(ptr)
        assert s.step_index == 2
        assert np.array_equal(s.field(), before)
        s.run(1)
        s.repartition(own1)
        s.run(2)
        s.synchronize()
        _check(oracle, s.field(), p, 5, "exact")
