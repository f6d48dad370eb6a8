"""pytest configuration: repo root on sys.path, the `gpu` marker, shared helpers."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REF_TESTS = os.path.join(ROOT, "tests", "golden", "reference_inputs")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run on the GPU box")


@pytest.fixture(scope="session", autouse=True)
def library_matches_tree():
    """Every test runs against a libnlh built from this checkout (its
    embedded build id equals the hash of the tree's library sources)."""
    import nonlocalheatequation_amd as N
    if os.path.exists(N.lib_path()):
        assert N.build_id() == N.source_build_id(), "libnlh.so is stale: rebuild with `make lib`"
    yield


def gpu_available() -> bool:
    try:
        import torch  # noqa: F401  (device counting only)
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.lib()
    return O


def read_input(name: str) -> str:
    with open(os.path.join(REF_TESTS, name)) as f:
        return f.read()


def virtual_peer_pairs(nx, ny, eps, tiles, owner, nranks, **kw) -> int:
    """(rank, peer) pairs with halo traffic over all ranks of a map: the
    nlh_info.npeers a solver running every rank (NLH_VIRTUAL_RANKS) reports."""
    import nonlocalheatequation_amd as N
    pairs = 0
    for r in range(nranks):
        lay = N.exchange_plan(nx, ny, eps, tiles, owner, r, nranks, **kw)
        pairs += len(set(int(p) for p in lay[:, 0]))
    return pairs


def _record_dir() -> str:
    d = os.path.join(os.environ.get("GRAFT_REPO_ROOT", ROOT), "gpurun_out")
    os.makedirs(d, exist_ok=True)
    return d


def check_l2(l2, l2_ref, u, u_ref, what: str = "") -> float:
    """The test-mode L2 criterion, recorded before it is asserted.

    |l2 - l2_ref| <= 1e-10 * max(l2_ref, floor), floor = n * (1e-12 * max|u_ref|)^2:
    1e-10 relative, except where the reference's own error_l2 sits below the
    L2 a field differing by the per-node tolerance everywhere would have (the
    rounding floor), where the bound is 1e-10 of that floor.  The observed
    relative difference, the exact Cauchy-Schwarz bound the measured per-node
    differences imply and the floor go to gpurun_out/parity_l2.jsonl.
    Returns the relative difference."""
    import json

    import numpy as np
    n = u_ref.size
    scale = float(np.max(np.abs(u_ref)))
    floor = n * (1e-12 * scale) ** 2
    dd = float(np.sum((np.asarray(u, dtype=np.float64) - u_ref) ** 2))
    cs = 2.0 * np.sqrt(l2_ref * dd) + dd  # |sum (e+d)^2 - sum e^2| <= 2 |e| |d| + |d|^2
    rel = abs(l2 - l2_ref) / l2_ref if l2_ref > 0 else abs(l2 - l2_ref)
    rec = {"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], "what": what, "n": n,
           "l2": l2, "l2_ref": l2_ref, "rel_diff": rel, "abs_diff": abs(l2 - l2_ref),
           "cauchy_schwarz_bound": cs, "floor": floor, "max_node_diff": float(np.max(np.abs(u - u_ref)))}
    try:
        with open(os.path.join(_record_dir(), "parity_l2.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")
    except OSError:
        pass
    assert abs(l2 - l2_ref) <= 1e-10 * max(l2_ref, floor), rec
    return rel
