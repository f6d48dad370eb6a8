"""CPU: the row-pair tap bookkeeping of k_pair_split and k_wide (nlh_pair.h
pair_shared / pair_scatter, nlh_wide.h wide_shared) restated in Python covers
the reference's disk exactly (src/2d_nonlocal_serial.cpp:256-270): with row A
skipping its shared taps and row B adding the pair sums, every output row
receives every (input row, level) term of the two rows once, for every
horizon the kernels are built for."""
import math
from collections import Counter

import pytest


def clen(eps: int, d: int) -> int:
    """Half-width of disk row d (the reference's (long)sqrt(eps^2 - d^2))."""
    return int(math.isqrt(eps * eps - d * d))


def pair_shared(eps: int, d: int) -> bool:
    """nlh_pair.h: output A + d takes level len(d) from row A and len(d-1)
    from row B; shared when the two are the same nonzero level."""
    return -eps < d <= eps and clen(eps, abs(d)) > 0 and clen(eps, abs(d)) == clen(eps, abs(d - 1))


def wide_shared(eps: int, dy: int) -> bool:
    """nlh_wide.h: output c + E - dy takes row c at dy and row c+1 at dy+1."""
    return -eps <= dy < eps and clen(eps, abs(dy)) > 0 and clen(eps, abs(dy)) == clen(eps, abs(dy + 1))


def direct_terms(eps: int, out_of):
    """(output, row, level) terms rows 0 and 1 contribute, one per disk row."""
    c = Counter()
    for r in (0, 1):
        for d in range(-eps, eps + 1):
            c[(out_of(r, d), r, clen(eps, abs(d)))] += 1
    return c


@pytest.mark.parametrize("eps", range(1, 65))
def test_pair_scatter_covers_disk(eps):
    # k_pair_split: row i adds H_len(d)(i) to output i + d
    got = Counter()
    for d in range(-eps, eps + 1):  # row A = 0
        if not pair_shared(eps, d):
            got[(d, 0, clen(eps, abs(d)))] += 1
    for d in range(-eps, eps + 1):  # row B = 1
        lv = clen(eps, abs(d))
        if pair_shared(eps, d + 1):  # the pair sum H_L(A) + H_L(B), same level
            assert clen(eps, abs(d + 1)) == lv
            got[(1 + d, 0, lv)] += 1
        got[(1 + d, 1, lv)] += 1
    assert got == direct_terms(eps, lambda r, d: r + d)


@pytest.mark.parametrize("eps", range(1, 65))
def test_wide_scatter_covers_disk(eps):
    # k_wide: row c adds H_len(dy)(c) to output c + E - dy
    got = Counter()
    for dy in range(-eps, eps + 1):  # row A = 0
        if not wide_shared(eps, dy):
            got[(eps - dy, 0, clen(eps, abs(dy)))] += 1
    for dy in range(-eps, eps + 1):  # row B = 1
        lv = clen(eps, abs(dy))
        if wide_shared(eps, dy - 1):
            assert clen(eps, abs(dy - 1)) == lv
            got[(1 + eps - dy, 0, lv)] += 1
        got[(1 + eps - dy, 1, lv)] += 1
    assert got == direct_terms(eps, lambda r, dy: r + eps - dy)


def test_shared_tap_counts():
    # E = 8 shares 6 taps (levels 6, 7), E = 32 shares 26
    assert [d for d in range(-8, 9) if pair_shared(8, d)] == [-4, -2, -1, 2, 3, 5]
    assert sum(wide_shared(32, dy) for dy in range(-32, 33)) == 26
    assert {clen(32, abs(dy)) for dy in range(-32, 33) if wide_shared(32, dy)} == {31, 30, 29, 28, 27, 24}
