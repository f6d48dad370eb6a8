"""CPU: the static partitioner (nlh_partition_tiles, recursive coordinate
bisection) and bin/2d_domain_decomposition, which replace the reference's
GMSH + METIS tool (src/domain_decomposition.cpp) and write the --file format
2d_nonlocal_distributed reads (write_mesh, :31-50).  Host-only: no GPU."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT

import nonlocalheatequation_amd as N

TOOL = os.path.join(ROOT, "bin", "2d_domain_decomposition")


def _connected(own, tx, ty, part):
    cells = {i for i in range(tx * ty) if own[i] == part}
    if not cells:
        return True
    seen, stack = set(), [next(iter(cells))]
    while stack:
        t = stack.pop()
        if t in seen:
            continue
        seen.add(t)
        x, y = t % tx, t // tx
        for nx, ny in ((x - 1, y), (x + 1, y), (x, y - 1), (x, y + 1)):
            if 0 <= nx < tx and 0 <= ny < ty and ny * tx + nx in cells:
                stack.append(ny * tx + nx)
    return seen == cells


@pytest.mark.parametrize("tx,ty,n", [(5, 5, 2), (5, 5, 4), (5, 5, 8), (4, 4, 3), (7, 3, 4), (16, 16, 8),
                                     (10, 1, 3), (2, 4, 8)])
def test_balanced_and_connected(tx, ty, n):
    own = N.partition_tiles((tx, ty), n)
    cnt = np.bincount(own, minlength=n)
    assert cnt.sum() == tx * ty and cnt.max() - cnt.min() <= 1
    assert all(_connected(own, tx, ty, p) for p in range(n))


def test_more_parts_than_tiles_and_single_part():
    own = N.partition_tiles((3, 1), 5)
    assert sorted(own.tolist()) == sorted(set(own.tolist())) and own.max() < 5
    assert not N.partition_tiles((4, 4), 1).any()


def test_weights_shift_the_cut():
    w = np.ones(16)
    w[:8] = 3.0  # top two rows (index gx + gy*4) three times as costly
    own = N.partition_tiles((4, 4), 2, w)
    load = [w[own == p].sum() for p in (0, 1)]
    assert abs(load[0] - load[1]) <= 3.0
    with pytest.raises(N.NLHError):
        N.partition_tiles((4, 4), 2, -w)


def test_partition_feeds_the_balancer():
    # a fresh partition is already a fixed point of the load balancer
    own = N.partition_tiles((5, 5), 4)
    cnt = np.bincount(own, minlength=4).astype(float)
    assert N.balance_owner((5, 5), 4, own, cnt)[0] == 0


def _run_tool(mesh, out, nodes, grains):
    p = subprocess.run([TOOL, mesh, str(out), str(nodes)], input="\n".join(map(str, grains)) + "\n",
                       capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    return p.stdout


def _read(path):
    tok = open(path).read().split()
    nx, ny, npx, npy, dh = int(tok[0]), int(tok[1]), int(tok[2]), int(tok[3]), float(tok[4])
    own = np.zeros(npx * npy, np.int32)
    rows = [tuple(map(int, tok[5 + 3 * i:8 + 3 * i])) for i in range(npx * npy)]
    for px, py, loc in rows:
        own[px + py * npx] = loc
    return nx, ny, npx, npy, dh, own, rows


def test_tool_writes_reference_format(tmp_path):
    out = tmp_path / "lb.txt"
    txt = _run_tool("400x400:0.0025", out, 4, [80, 80])
    assert "x dimension : 400\ny dimension : 400" in txt
    nx, ny, npx, npy, dh, own, rows = _read(out)
    assert (nx, ny, npx, npy, dh) == (80, 80, 5, 5, 0.0025)
    assert [r[:2] for r in rows] == [(i, j) for i in range(5) for j in range(5)]  # idx outer (:40-46)
    assert np.array_equal(own, N.partition_tiles((5, 5), 4))
    # the driver's reader takes it (tests/test_drivers.py runs such files on the GPU)
    assert open(out).read().splitlines()[0] == "80 80 5 5 0.0025"


def test_tool_single_node_and_bad_grain(tmp_path):
    out = tmp_path / "one.txt"
    _run_tool("40x20:0.05", out, 1, [10, 10])
    assert not _read(out)[5].any()
    txt = _run_tool("40x20:0.05", tmp_path / "bad.txt", 2, [7, 10])
    assert "not divisible" in txt and not (tmp_path / "bad.txt").exists()


def test_tool_reads_gmsh41(tmp_path):
    # a 4 x 2 quad mesh of spacing 0.5 in GMSH 4.1 ASCII
    nx, ny, h = 4, 2, 0.5
    tags = {}
    lines = []
    for j in range(ny + 1):
        for i in range(nx + 1):
            tags[(i, j)] = len(tags) + 1
            lines.append((i * h, j * h))
    quads = [(tags[(i, j)], tags[(i + 1, j)], tags[(i + 1, j + 1)], tags[(i, j + 1)])
             for j in range(ny) for i in range(nx)]
    msh = ["$MeshFormat", "4.1 0 8", "$EndMeshFormat", "$Nodes", f"1 {len(lines)} 1 {len(lines)}",
           f"2 1 0 {len(lines)}"]
    msh += [str(t) for t in range(1, len(lines) + 1)]
    msh += [f"{x} {y} 0" for x, y in lines]
    msh += ["$EndNodes", "$Elements", f"1 {len(quads)} 1 {len(quads)}", f"2 1 3 {len(quads)}"]
    msh += [f"{k + 1} {a} {b} {c} {d}" for k, (a, b, c, d) in enumerate(quads)]
    msh += ["$EndElements"]
    f = tmp_path / "m.msh"
    f.write_text("\n".join(msh) + "\n")
    out = tmp_path / "p.txt"
    txt = _run_tool(str(f), out, 2, [2, 1])
    assert "x dimension : 4\ny dimension : 2" in txt
    assert _read(out)[:5] == (2, 1, 2, 2, 0.5)
