"""CPU: the per-peer RCCL message layout nlh_create builds
(nlh_plan.cpp exchange_layout, read through nlh_exchange_plan) is
consistent between every sender and receiver -- what rank A packs for B,
piece for piece and offset for offset, is what B unpacks from A -- on the
BASELINE layouts: C3's 2 x 4 blocks, the reference's uneven 25s_8n map
(C5), the bench's 8-GPU weak-scaling layout, and horizons wider than a tile
(pieces from non-adjacent tiles).  The reference moves whole tiles with HPX
actions instead (src/2d_nonlocal_distributed.cpp:1121-1131,1156-1259)."""
import numpy as np
import pytest

from conftest import read_input

import nonlocalheatequation_amd as N


def _owner(name):
    tok = read_input(f"load_balance_{name}.txt").split()
    npx, npy = int(tok[2]), int(tok[3])
    own = [0] * (npx * npy)
    vals = list(map(int, tok[5:]))
    for i in range(npx * npy):
        px, py, loc = vals[3 * i:3 * i + 3]
        own[px + py * npx] = loc
    return (npx, npy), own, max(own) + 1


def _case(name):
    if name == "C3 2x4":
        return dict(nx=32768, ny=32768, eps=8, tiles=(2, 4), owner=None, nranks=8, split=False)
    if name == "C5 25s_8n":
        tiles, own, R = _owner("25s_8n")
        return dict(nx=46080, ny=46080, eps=8, tiles=tiles, owner=own, nranks=R, split=False)
    if name == "bench N=8 weak":
        return dict(nx=8192, ny=16384, eps=8, tiles=(2, 4), owner=None, nranks=8, split=False)
    if name == "eps > tile, split":
        return dict(nx=48, ny=32, eps=7, tiles=(6, 4), owner=None, nranks=5, split=True)
    if name == "eps > tile, 25s_4n":
        tiles, own, R = _owner("25s_4n")
        return dict(nx=40, ny=40, eps=9, tiles=tiles, owner=own, nranks=R, split=False)
    raise KeyError(name)


NAMES = ["C3 2x4", "C5 25s_8n", "bench N=8 weak", "eps > tile, split", "eps > tile, 25s_4n"]


@pytest.mark.parametrize("test", [False, True])
@pytest.mark.parametrize("name", NAMES)
def test_sender_layout_equals_receiver_layout(name, test):
    c = _case(name)
    R = c["nranks"]
    kw = dict(test=test, kernel="fast", dt=1e-7)
    lay = {r: N.exchange_plan(c["nx"], c["ny"], c["eps"], c["tiles"], c["owner"], r, R, c["split"], **kw)
           for r in range(R)}
    halo = N.halo_plan(c["nx"], c["ny"], c["eps"], c["tiles"], c["owner"], 0, R, c["split"], **kw)
    pairs = 0
    for a in range(R):
        la = lay[a]
        for b in range(R):
            if a == b:
                continue
            send = la[(la[:, 0] == b) & (la[:, 1] == 0)]
            lb = lay[b]
            recv = lb[(lb[:, 0] == a) & (lb[:, 1] == 1)]
            # piece, offset and rectangle, in message order
            assert np.array_equal(send[:, 2:], recv[:, 2:]), (name, a, b)
            if len(send):
                pairs += 1
                # the message is the pieces back to back
                sizes = send[:, 5] * send[:, 6]
                assert np.array_equal(send[:, 2], np.concatenate([[0], np.cumsum(sizes)[:-1]]))
    assert pairs > 0
    # every cross-rank piece of every destination appears once on each side
    for r in range(R):
        h = N.halo_plan(c["nx"], c["ny"], c["eps"], c["tiles"], c["owner"], r, R, c["split"], **kw)
        cross = h[h[:, 0] != h[:, 1]]
        recv = lay[r][lay[r][:, 1] == 1]
        got = sorted(map(tuple, recv[:, [0, 3, 4, 5, 6]].tolist()))
        want = sorted(map(tuple, cross[:, [0, 2, 3, 4, 5]].tolist()))
        assert got == want, (name, r)
    assert halo.shape[1] == 8


def test_c3_peer_count():
    # 2 x 4 blocks, 2*eps halo: corner ranks have 3 peers (side, side,
    # diagonal), the four inner ranks 5
    from conftest import virtual_peer_pairs
    assert virtual_peer_pairs(32768, 32768, 8, (2, 4), None, 8, dt=1e-7) == 32


def test_virtual_peer_pairs_counts_multi_peer():
    c = _case("C5 25s_8n")
    from conftest import virtual_peer_pairs
    n = virtual_peer_pairs(c["nx"], c["ny"], c["eps"], c["tiles"], c["owner"], c["nranks"], dt=1e-7)
    assert n > c["nranks"]  # several peers per rank: the grouped multi-peer exchange
