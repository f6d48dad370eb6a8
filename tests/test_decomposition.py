"""CPU: the multi-rank decomposition (block plan + halo plan of libnlh) run
with torch.distributed/gloo, world sizes 2 and 3.

Each rank owns the blocks nlh_block_plan() gives it, padded by an eps halo
(zero outside the domain), exchanges exactly the pieces nlh_halo_plan()
lists (gloo isend/irecv between ranks, copies within a rank), and steps its
blocks with a numpy restatement of sum_local in the reference's per-term
order.  After nt steps every owned node must equal the global oracle bit for
bit.  This is the GPU path's host logic (which pieces move where, blocks,
ownership maps incl. the reference's --file maps and eps > tile size) checked
without a GPU; tests/test_gpu_multiblock.py runs the same plans through the
HIP kernels.
"""
import os
import socket

import numpy as np
import pytest

from conftest import ROOT, read_input

import nonlocalheatequation_amd as N

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lens(eps):
    return [int(np.floor(np.sqrt(float(eps * eps - d * d)))) for d in range(eps + 1)]


def block_step(P, H, x0, y0, x1, y1, c2d, dh2, dt, lens, E):
    """sum_local (src/2d_nonlocal_serial.cpp:256-270) on the block-local
    rectangle [x0, x1) x [y0, y1) of a block padded by H, same per-term order:
    sx outer, sy inner, res += ((c*(u_j-u_i))*dh^2).  Needs H >= E beyond the
    rectangle."""
    u = P[H + y0:H + y1, H + x0:H + x1]
    res = np.zeros_like(u)
    for dx in range(-E, E + 1):
        ln = lens[abs(dx)]
        for dy in range(-ln, ln + 1):
            v = P[H + y0 + dy:H + y1 + dy, H + x0 + dx:H + x1 + dx]
            res += (c2d * (v - u)) * dh2
    return u + res * dt


def _worker(rank, world, port, case, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle as O
        nx, ny, eps, nt, tiles, owner, split = (case[k] for k in
                                                ("nx", "ny", "eps", "nt", "tiles", "owner", "split"))
        two = case.get("two_step", False)
        k, dh = 1.0, 1.0 / nx
        dt = eps ** 4 * dh * dh / (8 * k * N.disk_count(eps))
        p = O.params(nx, ny, eps, k, dt, dh, 0)
        u0 = O.test_init(p)
        ref = O.run(p, nt, u0)
        c2d = (k * 8) / (eps * dh) ** 4
        lens = _lens(eps)
        E = eps
        # the plans nlh_create builds: production fast mode (two steps per
        # pass, 2*eps halo) or the single-step exact kernel (eps halo)
        kern = "auto" if two else "exact"
        H = 2 * E if two else E
        kw = dict(k=k, dt=dt, dh=dh, test=False, kernel=kern)
        blocks = N.block_plan(nx, ny, eps, tiles, owner, world, split, **kw)
        allp = np.concatenate([N.halo_plan(nx, ny, eps, tiles, owner, r, world, split, **kw)
                               for r in range(world)] or [np.zeros((0, 8), np.int64)])
        # the plan's pieces fill exactly an H-wide frame (checked per piece below)
        for pc in allp:
            src, dst, gx0, gy0, w, h, sb, db = (int(v) for v in pc)
            _, _, bx0, by0, bw, bh = (int(v) for v in blocks[db])
            assert bx0 - H <= gx0 and gx0 + w <= bx0 + bw + H
            assert by0 - H <= gy0 and gy0 + h <= by0 + bh + H
        mine = {bi: b for bi, b in enumerate(blocks) if b[0] == rank}
        pad = {}
        for bi, b in mine.items():
            _, _, x0, y0, w, h = b
            P = np.zeros((h + 2 * H, w + 2 * H))
            P[H:H + h, H:H + w] = u0[y0:y0 + h, x0:x0 + w]
            pad[bi] = P

        def view(bi, gx0, gy0, w, h):
            _, _, x0, y0, _, _ = blocks[bi]
            return pad[bi][H + gy0 - y0:H + gy0 - y0 + h, H + gx0 - x0:H + gx0 - x0 + w]

        def exchange():
            reqs, recv = [], []
            for pc in allp:
                src, dst, gx0, gy0, w, h, sb, db = (int(v) for v in pc)
                if src == rank and dst != rank:
                    t = torch.from_numpy(np.ascontiguousarray(view(sb, gx0, gy0, w, h)))
                    reqs.append(dist.isend(t, dst))
                elif dst == rank and src != rank:
                    t = torch.empty((h, w), dtype=torch.float64)
                    reqs.append(dist.irecv(t, src))
                    recv.append((db, gx0, gy0, w, h, t))
                elif src == rank and dst == rank:
                    view(db, gx0, gy0, w, h)[...] = view(sb, gx0, gy0, w, h)
            for r in reqs:
                r.wait()
            for db, gx0, gy0, w, h, t in recv:
                view(db, gx0, gy0, w, h)[...] = t.numpy()

        t = 0
        while t < nt:
            exchange()
            steps = 2 if (two and nt - t >= 2) else 1
            new = {}
            for bi, b in mine.items():
                _, _, bx0, by0, w, h = (int(v) for v in b)
                if steps == 2:
                    # pass: u^{t+1} on the block + an E ring (inside the
                    # domain), then u^{t+2} on the block from it
                    ex0, ey0 = max(-E, -bx0), max(-E, -by0)
                    ex1, ey1 = min(w + E, nx - bx0), min(h + E, ny - by0)
                    Q = np.zeros_like(pad[bi])
                    Q[H + ey0:H + ey1, H + ex0:H + ex1] = block_step(pad[bi], H, ex0, ey0, ex1, ey1,
                                                                     c2d, dh * dh, dt, lens, E)
                    new[bi] = block_step(Q, H, 0, 0, w, h, c2d, dh * dh, dt, lens, E)
                else:
                    new[bi] = block_step(pad[bi], H, 0, 0, w, h, c2d, dh * dh, dt, lens, E)
            for bi, b in mine.items():
                pad[bi][H:H + int(b[5]), H:H + int(b[4])] = new[bi]
            t += steps
        ok, nblk = True, 0
        for bi, b in mine.items():
            _, _, x0, y0, w, h = (int(v) for v in b)
            ok &= bool(np.array_equal(pad[bi][H:H + h, H:H + w], ref[y0:y0 + h, x0:x0 + w]))
            nblk += 1
        q.put((rank, ok, nblk))
    finally:
        dist.destroy_process_group()


CASES = [
    dict(name="2x2 tiles locidx", nx=40, ny=60, eps=5, nt=4, tiles=(2, 2), owner=None, split=False, world=2),
    dict(name="4s_2n file map (L-shaped owner)", nx=40, ny=40, eps=3, nt=3, tiles=(2, 2),
         owner=[0, 1, 1, 1], split=False, world=2),
    dict(name="eps > tile, split tiles", nx=30, ny=20, eps=7, nt=2, tiles=(6, 4), owner=None, split=True, world=3),
    dict(name="25s_8n map folded to 3 ranks", nx=50, ny=50, eps=4, nt=3, tiles=(5, 5), owner="25s_8n",
         split=False, world=3),
    # bench.py --gpus 8 layout (decomposition(8) = 2x4 blocks, npx=2 npy=4, one per rank)
    dict(name="bench N=8 layout 2x4", nx=32, ny=64, eps=6, nt=3, tiles=(2, 4), owner=None, split=False, world=8),
    # the production two-step plan: 2*eps halo, one exchange per two steps
    # (odd nt: the last step single), as nlh_create builds it
    dict(name="two-step 2x2 locidx", nx=48, ny=40, eps=4, nt=5, tiles=(2, 2), owner=None, split=False,
         world=2, two_step=True),
    dict(name="two-step 25s_8n on 8 ranks", nx=50, ny=50, eps=3, nt=4, tiles=(5, 5), owner="25s_8n",
         split=False, world=8, two_step=True),
    dict(name="two-step eps > tile", nx=30, ny=24, eps=5, nt=4, tiles=(6, 4), owner=None, split=True,
         world=3, two_step=True),
]


def _owner_from_file(name, world):
    tok = read_input(f"load_balance_{name}.txt").split()
    npx, npy = int(tok[2]), int(tok[3])
    own = [0] * (npx * npy)
    vals = list(map(int, tok[5:]))
    for i in range(npx * npy):
        px, py, loc = vals[3 * i:3 * i + 3]
        own[px + py * npx] = loc % world
    return own


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_gloo_decomposition_bitwise(case):
    case = dict(case)
    if isinstance(case["owner"], str):
        case["owner"] = _owner_from_file(case["owner"], case["world"])
    world = case["world"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, case, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert sum(n for _, _, n in res) == len(N.block_plan(case["nx"], case["ny"], case["eps"], case["tiles"],
                                                          case["owner"], world, case["split"]))


def test_block_plan_covers_lattice():
    for tiles, owner, world, split in [((5, 5), None, 8, False), ((4, 3), None, 5, True),
                                       ((2, 2), [0, 1, 1, 1], 2, False)]:
        b = N.block_plan(100, 60, 5, tiles, owner, world, split)
        cover = np.zeros((60, 100), np.int32)
        for r, _, x0, y0, w, h in b:
            cover[y0:y0 + h, x0:x0 + w] += 1
        assert (cover == 1).all()


@pytest.mark.parametrize("kernel,test,width", [("exact", False, 1), ("exact", True, 1), ("auto", True, 2),
                                               ("auto", False, 2)])
def test_halo_plan_covers_halo_exactly(kernel, test, width):
    """The plan's pieces fill exactly the halo frame of each block: eps wide
    for the single-step kernels (exact), 2*eps for the two-step pass of the
    fast mode (production and test mode) -- the width nlh_create resolves."""
    nx, ny, eps, tiles, world = 60, 48, 7, (6, 4), 3
    kw = dict(k=1.0, dt=eps ** 4 / (nx * nx * 8.0 * N.disk_count(eps)), dh=1.0 / nx, test=test, kernel=kernel)
    H = width * eps
    b = N.block_plan(nx, ny, eps, tiles, None, world, True, **kw)
    for rank in range(world):
        pcs = N.halo_plan(nx, ny, eps, tiles, None, rank, world, True, **kw)
        for bi, blk in enumerate(b):
            if blk[0] != rank:
                continue
            _, _, x0, y0, w, h = blk
            need = np.zeros((ny, nx), np.int32)
            need[max(0, y0 - H):min(ny, y0 + h + H), max(0, x0 - H):min(nx, x0 + w + H)] = 1
            need[y0:y0 + h, x0:x0 + w] = 0
            got = np.zeros_like(need)
            for src, dst, gx0, gy0, pw, ph, sb, db in pcs:
                if db == bi:
                    got[gy0:gy0 + ph, gx0:gx0 + pw] += 1
                    sx0, sy0, sw, sh = b[sb][2:]
                    assert sx0 <= gx0 and gx0 + pw <= sx0 + sw and sy0 <= gy0 and gy0 + ph <= sy0 + sh
                    assert b[sb][0] == src and dst == rank
            assert np.array_equal(got, need)


@pytest.mark.parametrize("eps", [40, 64, 80, 150, 230])
def test_halo_width_large_horizons(eps):
    """Past the two-step horizons the fast kernels are single-step (k_wide to
    64, k_prefix_rt to 224, k_exact beyond): halo = eps, in every mode."""
    nx, ny, tiles, world = 600, 480, (3, 2), 2
    for test in (False, True):
        kw = dict(k=1.0, dt=eps ** 4 / (nx * nx * 8.0 * N.disk_count(eps)), dh=1.0 / nx, test=test, kernel="auto")
        b = N.block_plan(nx, ny, eps, tiles, None, world, True, **kw)
        pcs = N.halo_plan(nx, ny, eps, tiles, None, 0, world, True, **kw)
        assert len(pcs) > 0
        for src, dst, gx0, gy0, pw, ph, sb, db in pcs:
            x0, y0, w, h = b[db][2:]
            # every piece lies within eps of its destination block
            assert x0 - eps <= gx0 and gx0 + pw <= x0 + w + eps and y0 - eps <= gy0 and gy0 + ph <= y0 + h + eps
        assert max(max(x0 - p[2], p[2] + p[4] - (x0 + w), y0 - p[3], p[3] + p[5] - (y0 + h))
                   for p in pcs for (x0, y0, w, h) in [b[p[7]][2:]]) == eps


def test_default_owner_is_locidx():
    # locidx(): (i * nl) / (npx * npy)   src/2d_nonlocal_distributed.cpp:105-110
    o = N.resolve_owner(5, 5, 8)
    assert list(o) == [(i * 8) // 25 for i in range(25)]
    with pytest.raises(N.NLHError):
        N.resolve_owner(2, 2, 2, [0, 1, 2, 0])
