"""The separable form of the manufactured source's operator term, as the
fast test mode's L_h[W0] plane is computed from it (round 6: nlh_api.cpp
sep_tables + compute_lw, k_lw_sep; also nlh_pair.h OPT & 32768, harness
only): with the reference's zero-extended W0 = sx(x) sy(y)
(sum_local_test, src/2d_nonlocal_serial.cpp:235-252),

    L_h[W0](x, y) = c dh^2 (sum_l Sx'_l(x) Ty_l(y) + sx(x) Z(y)),

checked here on the CPU against the per-neighbour sum over the disk, at every
node of small lattices including the boundary band (tables restated in
numpy / long double exactly as sep_tables builds them)."""
import numpy as np
import pytest

import nonlocalheatequation_amd as N


def _lens(E):
    return [int(np.sqrt(float(E * E - d * d))) for d in range(E + 1)]


def _direct(nx, ny, E, dh, cd):
    lens = _lens(E)
    x = np.arange(nx)
    y = np.arange(ny)
    sx = np.sin(2 * np.pi * (x * dh))
    sy = np.sin(2 * np.pi * (y * dh))
    w = np.zeros((ny + 2 * E, nx + 2 * E))
    w[E:E + ny, E:E + nx] = np.outer(sy, sx)
    out = np.zeros((ny, nx))
    for dy in range(-E, E + 1):
        L = lens[abs(dy)]
        for dx in range(-L, L + 1):
            out += w[E + dy:E + dy + ny, E + dx:E + dx + nx] - w[E:E + ny, E:E + nx]
    return cd * out


def _separable(nx, ny, E, dh, cd):
    lens = _lens(E)
    lev = []
    prev = -1
    for d in range(E + 1):
        if lens[d] > 0 and lens[d] != prev:
            lev.append(lens[d])
        prev = lens[d]
    ld = np.longdouble
    def ext(n):
        v = np.zeros(n + 2 * E + 2, dtype=ld)
        v[E:E + n] = np.sin(2 * np.pi * (np.arange(n) * dh)).astype(ld)
        return v  # index g + E
    sxe, sye = ext(nx), ext(ny)
    disk = sum(2 * lens[abs(d)] + 1 for d in range(-E, E + 1))
    sxp = []
    for L in lev:
        s = sum(sxe[E + dx:E + dx + nx] for dx in range(-L, L + 1))
        sxp.append(cd * (s - (2 * L + 1) * sxe[E:E + nx]))
    sxr = cd * sxe[E:E + nx]
    ty = []
    for L in lev:
        ty.append(sum(sye[E + d:E + d + ny] for d in range(-E, E + 1) if lens[abs(d)] == L))
    z = -disk * sye[E:E + ny] + sum((2 * lens[abs(d)] + 1) * sye[E + d:E + d + ny] for d in range(-E, E + 1))
    # the tables are stored as doubles; the kernel forms the sum with fma
    sxp = [np.asarray(a, dtype=np.float64) for a in sxp]
    ty = [np.asarray(a, dtype=np.float64) for a in ty]
    out = np.outer(np.asarray(z, dtype=np.float64), np.asarray(sxr, dtype=np.float64))
    for a, b in zip(sxp, ty):
        out = out + np.outer(b, a)
    return out


@pytest.mark.parametrize("E,n", [(8, 96), (5, 61), (3, 40), (16, 130)])
def test_separable_source_matches_per_neighbour_sum(E, n):
    dh = 1.0 / n
    k = 1.0
    cd = (k * 8) / (E * dh) ** 4 * dh * dh
    a = _direct(n, n, E, dh, cd)
    b = _separable(n, n, E, dh, cd)
    scale = np.max(np.abs(a))
    assert np.max(np.abs(a - b)) <= 1e-12 * scale, (np.max(np.abs(a - b)), scale)
    assert N.disk_count(E) == sum(2 * l + 1 for l in [_lens(E)[abs(d)] for d in range(-E, E + 1)])
