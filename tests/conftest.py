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
