"""CPU: bench.py's launcher contract without a GPU.

* the block layouts per GPU count (1x1, 2x1, 2x2, 2x4: C3/C4/C5);
* ``--gpus N`` with WORLD_SIZE unset starts N rank processes itself; on a
  machine without a GPU every rank must fail loudly at nlh_create (no CPU
  fallback) and the launcher must exit non-zero instead of hanging.
"""
import os
import subprocess
import sys

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


def test_decomposition_layouts():
    assert [bench.decomposition(n) for n in (1, 2, 4, 8)] == [(1, 1), (2, 1), (2, 2), (2, 4)]
    for n in (3, 6, 16, 32):
        px, py = bench.decomposition(n)
        assert px * py == n and px <= py


def test_spawned_ranks_fail_loudly_without_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu-baseline"], env=env, capture_output=True, text=True,
                       timeout=240, cwd=ROOT)
    assert p.returncode != 0
    assert "no HIP device" in p.stderr, p.stderr[-2000:]
    assert '"metric"' not in p.stdout


def test_world_size_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 2 and "WORLD_SIZE" in p.stderr
