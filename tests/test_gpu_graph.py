"""GPU: production passes replayed from captured HIP graphs (NLH_GRAPH=1,
VERDICT r5 next 4) give the ungraphed path's field bit for bit.

Graphs hold the same kernels with the same arguments.  A single-stream
solver (one block) replays runs of 2..16 passes per hipGraphLaunch; solvers
with an exchange keep their passes ungraphed (nlh_api.cpp graph_passes:
multi-stream captures crashed intermittently on ROCm 7.2, DESIGN.md section
6) and must match too.  Call sequences mix graph runs with ungraphed
remainders and odd step counts; kernel timing brackets graph launches.
"""
import numpy as np
import pytest

import nonlocalheatequation_amd as N

pytestmark = pytest.mark.gpu

CASES = [
    # nx, ny, eps, tiles, split_tiles, extra environment
    (600, 500, 8, (1, 1), False, {}),
    (300, 240, 8, (3, 2), True, {}),
    (300, 240, 8, (3, 2), True, {"NLH_RCCL_SELF": "1"}),
    (512, 512, 8, (2, 4), False, {"NLH_VIRTUAL_RANKS": "8"}),
    (300, 240, 5, (3, 2), True, {"NLH_SCHED": "0"}),
    (300, 240, 5, (3, 2), True, {"NLH_SCHED": "1"}),
    (300, 240, 20, (3, 2), True, {}),   # k_wide: single-step passes
    (300, 240, 15, (2, 2), True, {}),   # k_fast: single-step passes
]
CALLS = [1, 7, 40, 33, 16]


def _run(monkeypatch, graph, nx, ny, eps, tiles, split, env, test=False, timing=False):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if graph:
        monkeypatch.setenv("NLH_GRAPH", "1")
    else:
        monkeypatch.delenv("NLH_GRAPH", raising=False)
    dh = 1.0 / nx
    dt = eps ** 4 * dh * dh / (8 * N.disk_count(eps))
    u0 = np.random.default_rng(eps).uniform(-1, 1, size=(ny, nx))
    steps = []
    with N.Solver(nx, ny, eps, 1.0, dt, dh, test=test, kernel="fast", tiles=tiles, split_tiles=split) as s:
        if test:
            s.test_init()
        else:
            s.input_init(u0)
        for n in CALLS:
            if timing:
                s.kernel_timing(True)
            s.run(n)
            s.synchronize()
            if timing:
                ms, st = s.kernel_time()
                steps.append(st)
                assert ms > 0
                s.kernel_timing(False)
        u = s.field()
        t = s.step_index
    for k in env:
        monkeypatch.delenv(k)
    return u, t, steps


@pytest.mark.parametrize("nx,ny,eps,tiles,split,env", CASES,
                         ids=[f"{c[0]}x{c[1]}-eps{c[2]}-{c[3][0]}x{c[3][1]}-{'-'.join(c[5]) or 'default'}"
                              for c in CASES])
def test_graph_bitwise(monkeypatch, nx, ny, eps, tiles, split, env):
    ref, t0, _ = _run(monkeypatch, False, nx, ny, eps, tiles, split, env)
    got, t1, _ = _run(monkeypatch, True, nx, ny, eps, tiles, split, env)
    assert t0 == t1 == sum(CALLS)
    assert np.array_equal(got.view(np.uint64), ref.view(np.uint64)), np.max(np.abs(got - ref))


def test_graph_with_kernel_timing(monkeypatch):
    """Kernel timing 1 brackets graph launches like pass launches: the same
    step counts, the same field."""
    ref, _, s0 = _run(monkeypatch, False, 300, 240, 8, (3, 2), True, {"NLH_RCCL_SELF": "1"}, timing=True)
    got, _, s1 = _run(monkeypatch, True, 300, 240, 8, (3, 2), True, {"NLH_RCCL_SELF": "1"}, timing=True)
    assert s0 == s1 == CALLS
    assert np.array_equal(got, ref)


def test_graph_off_in_test_mode(monkeypatch):
    """Test mode keeps the ungraphed passes (the source constants change per
    step): NLH_GRAPH=1 changes nothing there."""
    ref, _, _ = _run(monkeypatch, False, 300, 240, 8, (3, 2), True, {}, test=True)
    got, _, _ = _run(monkeypatch, True, 300, 240, 8, (3, 2), True, {}, test=True)
    assert np.array_equal(got, ref)
