"""CPU: the load-balancing policy (nlh_balance_owner, host-only) that replaces
the reference's idle-rate driven work_realloc + DFS/BFS tile migration
(src/2d_nonlocal_distributed.cpp:844-959), on the reference's own partition
maps (tests/load_balance_*.txt), and the multi-rank round with
torch.distributed/gloo (busy times all-gathered, every rank derives the same
map, moved tiles shipped rank to rank)."""
import os
import socket

import numpy as np
import pytest

from conftest import read_input

import nonlocalheatequation_amd as N

MAPS = ["load_balance_4s_2n.txt", "load_balance_25s_2n.txt", "load_balance_25s_4n.txt",
        "load_balance_25s_8n.txt"]


def _map(name):
    tok = read_input(name).split()
    npx, npy = int(tok[2]), int(tok[3])
    own = np.zeros(npx * npy, np.int32)
    vals = list(map(int, tok[5:]))
    for i in range(npx * npy):
        px, py, loc = vals[3 * i:3 * i + 3]
        own[px + py * npx] = loc
    return npx, npy, own, int(own.max()) + 1


def _converge(tiles, R, own, cost, rounds=12):
    """Balancing rounds with busy = tiles owned x per-tile cost of the rank."""
    hist = []
    for _ in range(rounds):
        busy = np.bincount(own, minlength=R) * np.asarray(cost, float)
        moved, own = N.balance_owner(tiles, R, own, busy)
        hist.append(moved)
        if moved == 0:
            break
    return own, hist


@pytest.mark.parametrize("name", MAPS)
def test_reference_maps_even_out(name):
    npx, npy, own, R = _map(name)
    new, hist = _converge((npx, npy), R, own, [1.0] * R)
    cnt = np.bincount(new, minlength=R)
    assert hist[-1] == 0 and len(hist) <= 4
    assert cnt.min() >= 1
    assert cnt.max() - cnt.min() <= 1, cnt
    # a balanced map is a fixed point
    assert N.balance_owner((npx, npy), R, new, cnt.astype(float))[0] == 0


def test_25s_4n_single_round():
    npx, npy, own, R = _map("load_balance_25s_4n.txt")
    cnt = np.bincount(own, minlength=R)
    moved, new = N.balance_owner((npx, npy), R, own, cnt.astype(float))
    assert moved == int(np.abs(np.bincount(new, minlength=R) - cnt).sum() // 2) > 0
    # every moved tile went from a rank above the mean to one below it
    mean = cnt.mean()
    for t in np.nonzero(new != own)[0]:
        assert cnt[own[t]] > mean > cnt[new[t]]


def test_heterogeneous_ranks_converge_to_speed_ratio():
    # 16 tiles over 2 ranks, rank 0 three times slower per tile: 4 / 12
    own = np.array([0] * 8 + [1] * 8, np.int32)
    new, hist = _converge((4, 4), 2, own, [3.0, 1.0])
    assert list(np.bincount(new, minlength=2)) == [4, 12]
    assert hist[-1] == 0


def test_dead_band_and_odd_counts_do_not_flip():
    # 13 / 12 tiles at equal speed: the reference's quota (+-1) would flip a
    # tile every round; the predicted-time guard keeps the map
    own = np.array([(i * 2) // 25 for i in range(25)], np.int32)
    assert N.balance_owner((5, 5), 2, own, np.array([13.0, 12.0]))[0] == 0
    # within the 0.3-tile dead band: no quota at all
    assert N.balance_owner((5, 5), 2, own, np.array([12.6, 12.4]))[0] == 0


def test_idle_rank_receives_work_and_donors_keep_one_tile():
    own = np.zeros(9, np.int32)
    own[8] = 1  # rank 2 owns nothing
    moved, new = N.balance_owner((3, 3), 3, own, np.array([8.0, 1.0, 0.0]))
    cnt = np.bincount(new, minlength=3)
    assert moved > 0 and cnt.min() >= 1


def test_zero_busy_and_bad_arguments():
    own = np.array([0, 0, 1, 1], np.int32)
    assert N.balance_owner((2, 2), 2, own, np.zeros(2)) == (0, pytest.approx(own))
    with pytest.raises(N.NLHError):
        N.balance_owner((2, 2), 2, np.array([0, 0, 1, 2], np.int32), np.ones(2))
    with pytest.raises(N.NLHError):
        N.balance_owner((2, 2), 2, own, np.array([1.0, -1.0]))


def test_deterministic():
    npx, npy, own, R = _map("load_balance_25s_8n.txt")
    busy = np.random.default_rng(5).uniform(1, 3, R)
    a = N.balance_owner((npx, npy), R, own, busy)
    b = N.balance_owner((npx, npy), R, own.copy(), busy.copy())
    assert a[0] == b[0] and np.array_equal(a[1], b[1])


# ---- world-size-2/3 round with gloo -----------------------------------------
torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, name, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        npx, npy, own, R = _map(name)
        own = own % world
        tw = th = 6
        rng = np.random.default_rng(11)
        field = rng.standard_normal((npy * th, npx * tw))  # same on every rank
        tiles = {t: field[(t // npx) * th:(t // npx + 1) * th, (t % npx) * tw:(t % npx + 1) * tw].copy()
                 for t in range(npx * npy) if own[t] == rank}
        # this rank's busy time: its tiles x a rank-dependent per-tile cost
        mine = torch.tensor([len(tiles) * (1.0 + 0.5 * rank)], dtype=torch.float64)
        allb = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(allb, mine)
        busy = np.array([float(b) for b in allb])
        moved, new = N.balance_owner((npx, npy), world, own, busy)
        maps = [torch.zeros(npx * npy, dtype=torch.int32) for _ in range(world)]
        dist.all_gather(maps, torch.from_numpy(new.copy()))
        same = all(np.array_equal(m.numpy(), new) for m in maps)
        # ship moved tiles (tile order per peer), as nlh_repartition does
        reqs = []
        for t in range(npx * npy):
            if own[t] == rank and new[t] != rank:
                reqs.append(dist.isend(torch.from_numpy(tiles.pop(t)), int(new[t])))
        for t in range(npx * npy):
            if new[t] == rank and own[t] != rank:
                buf = torch.zeros((th, tw), dtype=torch.float64)
                dist.recv(buf, int(own[t]))
                tiles[t] = buf.numpy()
        for r in reqs:
            r.wait()
        ok = set(tiles) == {t for t in range(npx * npy) if new[t] == rank}
        for t, a in tiles.items():
            ok &= np.array_equal(a, field[(t // npx) * th:(t // npx + 1) * th, (t % npx) * tw:(t % npx + 1) * tw])
        q.put((rank, bool(same), bool(ok), int(moved)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name", [(2, "load_balance_25s_2n.txt"), (3, "load_balance_25s_4n.txt")])
def test_gloo_balance_round(world, name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(r[1] and r[2] for r in res), res
    assert len({r[3] for r in res}) == 1


def test_fallback_moves_the_donor_tile_nearest_the_receiver():
    """No donor tile borders a receiver (a neutral rank sits between them):
    the policy's fallback moves the donor tile nearest (Manhattan; the BFS
    distance map of nlh_plan.cpp) to the receiver's tiles, lowest index first
    on ties; deterministic."""
    # 6 x 1: receiver 0 | neutral 1 | donor 2 x 4
    moved, new = N.balance_owner((6, 1), 3, np.array([0, 1, 2, 2, 2, 2], np.int32), [1.0, 17.0, 33.0])
    assert moved == 2 and new.tolist() == [0, 1, 0, 0, 2, 2]
    # 5 x 5: receiver in one corner, donor block in the far corner, neutral between
    tx = ty = 5
    own = np.ones(tx * ty, np.int32)
    own[0] = 0
    for gy in range(3, 5):
        for gx in range(3, 5):
            own[gx + gy * tx] = 2
    busy = [1.0, 20.5, 40.0]  # rank 1 exactly at the mean: neither donor nor receiver
    moved, new = N.balance_owner((tx, ty), 3, own, busy)
    assert moved >= 1
    got = [t for t in range(tx * ty) if own[t] == 2 and new[t] == 0]
    # the donor tile nearest tile 0 (Manhattan), lowest index on ties: (3, 3)
    dist = {t: (t % tx) + (t // tx) for t in range(tx * ty) if own[t] == 2}
    first = min(dist, key=lambda t: (dist[t], t))
    assert first in got
    again = N.balance_owner((tx, ty), 3, own, busy)
    assert again[0] == moved and np.array_equal(again[1], new)
