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
