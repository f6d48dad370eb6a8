"""GPU: the multi-block step (halo pieces, interior/boundary-band split,
overlapped exchange stream) through the C ABI, on one MI355X.

split_tiles=True keeps every tile as its own device block, so one rank runs
the same halo machinery a multi-GPU run uses (local block-to-block copies in
place of RCCL send/recv).  Exact kernel: bitwise vs the oracle; fast kernel:
1e-12 of field scale.  The last test runs two RCCL ranks as two processes;
RCCL refuses two ranks on one device, in which case it is skipped (the
RCCL path then runs in the driver's multi-GPU bench; its plan is covered on
CPU by tests/test_decomposition.py).
"""
import multiprocessing as mp
import os

import numpy as np
import pytest

from conftest import check_nodes, virtual_peer_pairs

import nonlocalheatequation_amd as N

pytestmark = pytest.mark.gpu


def _run(nx, ny, eps, nt, test, kernel, tiles, split, owner=None, k=1.0, dt=None, dh=None, u0=None):
    dh = dh or 1.0 / nx
    dt = dt or eps ** 4 * dh * dh / (8 * k * N.disk_count(eps))
    with N.Solver(nx, ny, eps, k, dt, dh, test=test, kernel=kernel, tiles=tiles,
                  split_tiles=split, owner=owner) as s:
        if u0 is None:
            s.test_init()
        else:
            s.input_init(u0)
        s.run(nt)
        s.synchronize()
        return s.field(), s.errors(nt), s.info(), (k, dt, dh)


CASES = [
    (64, 48, 5, 6, (2, 2)),
    (30, 20, 7, 3, (6, 4)),      # eps > tile size: pieces from non-adjacent tiles
    (512, 384, 8, 4, (4, 3)),    # 128x128 tiles: full strips + bands in the fast kernel
    (300, 200, 3, 5, (3, 2)),
]


@pytest.mark.parametrize("nx,ny,eps,nt,tiles", CASES)
def test_split_tiles_exact_bitwise(oracle, nx, ny, eps, nt, tiles):
    u, (l2, li), info, (k, dt, dh) = _run(nx, ny, eps, nt, True, "exact", tiles, True)
    assert info.nblocks == tiles[0] * tiles[1]
    p = oracle.params(nx, ny, eps, k, dt, dh, 1)
    ref = oracle.run(p, nt)
    assert np.array_equal(u, ref)
    assert li == oracle.errors(p, nt, ref)[1]


@pytest.mark.parametrize("nx,ny,eps,nt,tiles", CASES)
def test_split_tiles_fast(oracle, nx, ny, eps, nt, tiles):
    rng = np.random.default_rng(7)
    u0 = rng.uniform(-1, 1, size=(ny, nx))
    u, _, info, (k, dt, dh) = _run(nx, ny, eps, nt, False, "fast", tiles, True, u0=u0)
    assert info.kernel == N.KERNEL_FAST
    p = oracle.params(nx, ny, eps, k, dt, dh, 0)
    ref = oracle.run(p, nt, u0)
    check_nodes(u, ref)


def test_merged_vs_split_consistent():
    a = _run(256, 256, 6, 5, False, "fast", (4, 4), False)[0]
    b = _run(256, 256, 6, 5, False, "fast", (4, 4), True)[0]
    # the fast kernel's row order (sweep direction alternates per segment)
    # follows the blocking, so results agree to summation rounding only
    assert np.max(np.abs(a - b)) <= 1e-13 * np.max(np.abs(a))
    ea = _run(256, 256, 6, 5, False, "exact", (4, 4), False)[0]
    eb = _run(256, 256, 6, 5, False, "exact", (4, 4), True)[0]
    assert np.array_equal(ea, eb)  # the parity kernel is blocking-independent


def test_single_rank_owner_map_from_file(oracle):
    # tests/load_balance_4s_2n.txt: 20x20 tiles, 2x2, dh=0.0025; all tiles on one GPU
    nx = ny = 40
    u, (l2, li), info, _ = _run(nx, ny, 5, 10, True, "exact", (2, 2), False, owner=[0, 0, 0, 0],
                                k=1.0, dt=0.0005, dh=0.0025)
    p = oracle.params(nx, ny, 5, 1.0, 0.0005, 0.0025, 1)
    assert np.array_equal(u, oracle.run(p, 10))


def _rccl_rank(rank, idq, q):
    try:
        import torch
        ndev = max(1, torch.cuda.device_count())  # counting only: no GPU init
        # rank 0 makes the RCCL unique id and hands it to rank 1; the parent
        # process never touches RCCL (an unused id's bootstrap root thread
        # would outlive the test in it)
        if rank == 0:
            cid = N.comm_unique_id()
            idq.put(cid)
        else:
            cid = idq.get(timeout=120)
        nx = ny = 256
        eps = 8
        dh = 1.0 / nx
        dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
        with N.Solver(nx, ny, eps, 1.0, dt, dh, test=False, kernel="fast", device=rank % ndev, rank=rank,
                      nranks=2, tiles=(2, 1), comm_id=cid) as s:
            s.test_init()
            s.run(5)
            s.synchronize()
            u = s.gather(0)
            l2, li = s.errors(5)
            q.put((rank, "ok", (u if rank == 0 else None, li), ndev))
    except Exception as e:  # noqa: BLE001
        q.put((rank, "err", str(e), locals().get("ndev", 1)))


def test_rccl_two_ranks(oracle):
    """Two RCCL ranks (two processes): the cross-rank halo exchange, the
    gather and the all-reduced norms.  On a one-GPU box both ranks land on
    device 0, which RCCL refuses at communicator creation ("Duplicate GPU
    detected", ncclInvalidUsage from ncclCommInitRank) -- only that exact
    refusal is a skip; any other failure (e.g. in the grouped send/recv) fails."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    idq = ctx.Queue()
    ps = [ctx.Process(target=_rccl_rank, args=(r, idq, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    ndev = 1
    try:
        for _ in range(2):
            r, st, v, nd = q.get(timeout=180)
            res[r] = (st, v)
            ndev = nd
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errs = [v for st, v in res.values() if st == "err"]
    if errs:
        refused = all(e.startswith("nlh_create failed") and "ncclCommInitRank" in e and "invalid usage" in e
                      for e in errs)
        if ndev == 1 and refused:
            pytest.skip(f"one GPU: RCCL refuses two ranks on one device ({errs[0][:120]})")
        pytest.fail(str(errs))
    nx = 256
    dh = 1.0 / nx
    dt = 8 ** 4 * dh * dh / (8 * N.disk_count(8))
    p = oracle.params(nx, nx, 8, 1.0, dt, dh, 0)
    ref = oracle.run(p, 5)
    u = res[0][1][0]
    check_nodes(u, ref)
    li_ref = oracle.errors(p, 5, ref)[1]
    assert res[0][1][1] == res[1][1][1]  # the all-reduced max is the same on both ranks
    assert abs(res[0][1][1] - li_ref) <= 1e-12 * li_ref


@pytest.mark.parametrize("kernel,test,eps,nt", [("exact", True, 5, 6), ("fast", False, 8, 6),
                                                ("fast", False, 8, 5), ("fast", True, 6, 4),
                                                ("fast", False, 20, 3), ("fast", True, 32, 2)])
def test_rccl_self_transport(oracle, monkeypatch, kernel, test, eps, nt):
    """NLH_RCCL_SELF: one rank with a size-1 RCCL communicator; every halo
    piece between its blocks is packed, sent with ncclSend/ncclRecv to self
    and unpacked -- the multi-GPU transport, on one MI355X."""
    monkeypatch.setenv("NLH_RCCL_SELF", "1")
    nx, ny, tiles = 384, 256, (3, 2)
    rng = np.random.default_rng(5)
    u0 = None if test else rng.uniform(-1, 1, size=(ny, nx))
    u, (l2, li), info, (k, dt, dh) = _run(nx, ny, eps, nt, test, kernel, tiles, True, u0=u0)
    assert info.nblocks == 6 and info.npeers == 1 and info.halo_bytes_sent > 0
    p = oracle.params(nx, ny, eps, k, dt, dh, int(test))
    ref = oracle.run(p, nt, u0)
    if kernel == "exact":
        assert np.array_equal(u, ref)
        assert li == oracle.errors(p, nt, ref)[1]
    else:
        check_nodes(u, ref)


@pytest.mark.parametrize("kernel,test", [("exact", True), ("fast", False), ("fast", True)])
def test_forced_band_schedule_matches_oracle(oracle, monkeypatch, kernel, test):
    """NLH_FORCE_BANDS runs one block through the multi-GPU schedule (interior
    kernel, then the halo bands on their own stream with short segments)."""
    monkeypatch.setenv("NLH_FORCE_BANDS", "1")
    rng = np.random.default_rng(11)
    nx, ny, eps, nt = 400, 300, 8, 5
    u0 = rng.uniform(-1, 1, size=(ny, nx))
    u, _, info, (k, dt, dh) = _run(nx, ny, eps, nt, test, kernel, (1, 1), False, u0=u0)
    ref = oracle.run(oracle.params(nx, ny, eps, k, dt, dh, int(test)), nt, u0)
    if kernel == "exact":
        assert np.array_equal(u, ref)
    else:
        check_nodes(u, ref)


@pytest.mark.parametrize("tiles,split,kernel", [((1, 1), False, "exact"), ((3, 2), True, "exact"),
                                                ((2, 2), True, "fast")])
def test_snapshot_overlaps_later_steps(oracle, tiles, split, kernel):
    """nlh_snapshot_begin after step n, more steps enqueued behind it, then
    nlh_snapshot_wait: the snapshot is u(n), the field u(n + m)."""
    nx, ny, eps, n, m = 192, 128, 6, 5, 4
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    p = oracle.params(nx, ny, eps, 1.0, dt, dh, 1)
    with N.Solver(nx, ny, eps, 1.0, dt, dh, test=True, kernel=kernel, tiles=tiles, split_tiles=split) as s:
        s.test_init()
        s.run(n)
        s.snapshot_begin()
        with pytest.raises(N.NLHError):
            s.snapshot_begin()  # one snapshot in flight
        s.run(m)
        snap = s.snapshot_wait()
        u = s.field()
    for got, t in ((snap, n), (u, n + m)):
        ref = oracle.run(p, t)
        if kernel == "exact":
            assert np.array_equal(got, ref)
        else:
            check_nodes(got, ref)


def _owner_25s_8n():
    from conftest import virtual_peer_pairs, read_input
    tok = read_input("load_balance_25s_8n.txt").split()
    npx, npy = int(tok[2]), int(tok[3])
    own = [0] * (npx * npy)
    vals = list(map(int, tok[5:]))
    for i in range(npx * npy):
        px, py, loc = vals[3 * i:3 * i + 3]
        own[px + py * npx] = loc
    return own


@pytest.mark.parametrize("kernel,test,nt", [("exact", True, 5), ("fast", False, 5), ("fast", True, 4)])
def test_virtual_ranks_uneven_map(oracle, monkeypatch, kernel, test, nt):
    """NLH_VIRTUAL_RANKS=8 with the reference's uneven 25-tile / 8-owner map
    (tests/load_balance_25s_8n.txt): each owner's tiles merged into its own
    blocks as on its own GPU, pieces between owners packed and sent over RCCL
    (to self), pieces inside an owner copied -- the multi-rank message
    pattern of C5's uneven case on one MI355X."""
    monkeypatch.setenv("NLH_VIRTUAL_RANKS", "8")
    owner = _owner_25s_8n()
    nx = ny = 5 * 48
    eps = 6
    rng = np.random.default_rng(25)
    u0 = None if test else rng.uniform(-1, 1, size=(ny, nx))
    u, (l2, li), info, (k, dt, dh) = _run(nx, ny, eps, nt, test, kernel, (5, 5), False, owner=owner, u0=u0)
    plan = N.block_plan(nx, ny, eps, (5, 5), owner, 8, False)
    # every virtual rank with its own per-peer buffers: the grouped multi-peer exchange
    pairs = virtual_peer_pairs(nx, ny, eps, (5, 5), owner, 8, test=test, kernel=kernel, k=k, dt=dt, dh=dh)
    assert info.nblocks == len(plan) > 8 and info.npeers == pairs > 8 and info.halo_bytes_sent > 0
    p = oracle.params(nx, ny, eps, k, dt, dh, int(test))
    ref = oracle.run(p, nt, u0)
    if kernel == "exact":
        assert np.array_equal(u, ref)
        assert li == oracle.errors(p, nt, ref)[1]
    else:
        check_nodes(u, ref)


@pytest.mark.parametrize("kernel,test", [("exact", True), ("fast", True), ("fast", False)])
@pytest.mark.parametrize("root", [0, 3])
def test_virtual_ranks_gather_and_errors(oracle, monkeypatch, kernel, test, root):
    """Under NLH_VIRTUAL_RANKS every rank's blocks travel to the root over
    RCCL (to self) in its own plan-ordered message, as nlh_gather_field does
    between real ranks (the reference pulls every tile to locality 0,
    src/2d_nonlocal_distributed.cpp:496,1121-1131); the error norms are summed
    per rank first, then over ranks (:495-520)."""
    monkeypatch.setenv("NLH_VIRTUAL_RANKS", "8")
    owner = _owner_25s_8n()
    nx = ny = 5 * 40
    eps, nt = 5, 5
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    with N.Solver(nx, ny, eps, 1.0, dt, dh, test=test, kernel=kernel, tiles=(5, 5), owner=owner) as s:
        s.test_init()
        s.run(nt)
        s.synchronize()
        u = s.field()
        g = s.gather(root)
        l2, li = s.errors(nt)
        assert s.info().owners == 8
    assert np.array_equal(g, u)
    p = oracle.params(nx, ny, eps, 1.0, dt, dh, int(test))
    ref = oracle.run(p, nt)
    rl2, rli = oracle.errors(p, nt, ref)
    if kernel == "exact":
        assert np.array_equal(u, ref) and li == rli
        assert l2 == pytest.approx(rl2, rel=1e-13)
    else:
        check_nodes(u, ref)
        if test:
            assert l2 == pytest.approx(rl2, rel=1e-10)
