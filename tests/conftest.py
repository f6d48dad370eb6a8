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

    The per-node differences d (each asserted <= 1e-12 of field scale by the
    caller) bound how far the L2 can move: |l2 - l2_ref| <= 2 sqrt(l2_ref sum d^2)
    + sum d^2 (Cauchy-Schwarz).  The regime follows that bound:
    * 1e-10 relative, where the bound itself is below 1e-10 of l2_ref -- the
      per-node agreement leaves no room for more, so the L2 must match to that;
    * the bound itself, where it exceeds 1e-10 of l2_ref: a few-ulp per-node
      difference can then move the L2 by more than 1e-10 relative (the
      reference's own error is at the rounding floor of the field: C4's 100
      steps, 3.6e-10 rms per node, give 6.5e-6 relative from 1.2e-15 rms
      differences; k_prefix_rt's eps 65-130 runs 1.1-4.8e-10 relative from
      <= 1.5e-13 per node).  This is AUTO's test-mode L2 contract there
      (include/nlh.h): 1e-10 relative only where the
      reference's error is above the rounding floor of the node differences;
    * always: the L2 difference is the one the measured d imply (within the
      bound above plus 1e-13 of l2_ref for the two reductions' own rounding)
      -- the norm kernel adds nothing of its own.  (Round 4 asserted a fixed
      1e-10 absolute in the second regime, vacuous for l2_ref < 1e-10.)
    The observed relative difference, the bound and the regime go to
    gpurun_out/parity_l2.jsonl.  Returns the relative difference."""
    import json

    import numpy as np
    n = u_ref.size
    scale = float(np.max(np.abs(u_ref)))
    dd = float(np.sum((np.asarray(u, dtype=np.float64) - u_ref) ** 2))
    cs = 2.0 * np.sqrt(l2_ref * dd) + dd
    diff = abs(l2 - l2_ref)
    rel = diff / l2_ref if l2_ref > 0 else diff
    relative = cs <= 1e-10 * l2_ref
    rec = {"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], "what": what, "n": n,
           "l2": l2, "l2_ref": l2_ref, "rel_diff": rel, "abs_diff": diff, "cauchy_schwarz_bound": cs,
           "error_per_node_rms": float(np.sqrt(l2_ref / n)), "field_scale": scale,
           "criterion": "1e-10 relative" if relative else "Cauchy-Schwarz bound (rounding floor: bound > 1e-10 relative)",
           "max_node_diff": float(np.max(np.abs(u - u_ref)))}
    try:
        with open(os.path.join(_record_dir(), "parity_l2.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")
    except OSError:
        pass
    if relative:
        assert diff <= 1e-10 * l2_ref, rec
    assert diff <= cs * (1 + 1e-9) + 1e-13 * l2_ref, rec
    return rel


def node_errors(u, u_ref, scale=None, rows=2048) -> dict:
    """Per-node error statistics of u against u_ref, chunked over rows so
    full-size fields need no full-size temporaries: the max absolute
    difference, the field scale (max |u_ref| unless given), and north_star's
    per-node RELATIVE error |u - u_ref| / |u_ref| -- its maximum over the nodes
    with |u_ref| >= 1e-6 and >= 1e-3 of the scale (near the field's zero
    crossings a relative error says nothing: a node's rounding follows the
    magnitude of the neighbours it sums, not its own) and the fraction of
    those nodes within 1e-12 relative."""
    import numpy as np
    a = np.asarray(u, dtype=np.float64)
    b = np.asarray(u_ref, dtype=np.float64)
    a2 = a.reshape(a.shape[0], -1) if a.ndim > 1 else a.reshape(1, -1)
    b2 = b.reshape(b.shape[0], -1) if b.ndim > 1 else b.reshape(1, -1)
    sc = float(np.max(np.abs(b))) if scale is None else float(scale)
    dmax = 0.0
    rel6 = rel3 = 0.0
    n6 = ok6 = 0
    for y in range(0, a2.shape[0], rows):
        x = a2[y:y + rows]
        r = b2[y:y + rows]
        d = np.abs(x - r)
        dmax = max(dmax, float(np.max(d)) if d.size else 0.0)
        ar = np.abs(r)
        m6 = ar >= 1e-6 * sc
        if np.any(m6):
            q = d[m6] / ar[m6]
            rel6 = max(rel6, float(np.max(q)))
            n6 += int(q.size)
            ok6 += int(np.count_nonzero(q <= 1e-12))
        m3 = ar >= 1e-3 * sc
        if np.any(m3):
            rel3 = max(rel3, float(np.max(d[m3] / ar[m3])))
    return {"max_abs_diff": dmax, "field_scale": sc, "max_rel_node_1e-6": rel6, "max_rel_node_1e-3": rel3,
            "nodes_1e-6": n6, "frac_nodes_rel_le_1e-12": (ok6 / n6) if n6 else 1.0}


def check_nodes(u, u_ref, what: str = "", scale=None, tol: float = 1e-12) -> dict:
    """The per-node criterion of every FAST kernel: |u - u_ref|
    <= tol * field scale at every node, asserted; north_star's per-node
    relative error (node_errors) recorded beside it, before the assertion, to
    gpurun_out/parity_nodes.jsonl."""
    import json
    import numpy as np
    st = node_errors(u, u_ref, scale)
    rec = {"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0], "what": what,
           "n": int(getattr(u_ref, "size", 0)), "tol_field_scale": tol, **st}
    if scale is not None:  # the scale given (e.g. the run's largest field): the final field's beside it
        fin = float(np.max(np.abs(u_ref)))
        rec["final_field_scale"] = fin
        rec["max_abs_diff_over_final_scale"] = st["max_abs_diff"] / fin if fin > 0 else None
    try:
        with open(os.path.join(_record_dir(), "parity_nodes.jsonl"), "a") as f:
            f.write(json.dumps(rec) + "\n")
    except OSError:
        pass
    assert st["max_abs_diff"] <= tol * st["field_scale"], rec
    return st
