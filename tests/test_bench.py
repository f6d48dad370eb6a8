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
    assert '"value"' not in p.stdout  # no result line: only the error line (round 5)


def test_world_size_mismatch_is_an_error():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert p.returncode == 2 and "WORLD_SIZE" in p.stderr


def test_multi_gpu_line_fields():
    """The N > 1 line carries RCCL's own rank count, the per-pass exchange
    report (max over ranks) and, with --strong, T1 / (N T_N)."""
    phases = {"wall_ms": 100.0, "interior_ms": 80.0, "band_ms": 12.0, "exchange_ms": 30.0,
              "exposed_exchange_ms": 20.0, "passes": 50, "steps": 100, "halo_bytes_sent": 3_145_728}
    t1 = {"ms_per_step": 16.0, "value": 67.1, "build_id": "x", "kernel_avg_us": 3200.0}
    f = bench.scaling_fields(8, True, 2.5, t1=t1, phases=phases, comm_seen=8)
    assert f["nranks_seen"] == 8
    assert f["strong_efficiency"] == 16.0 / (8 * 2.5)
    assert f["strong_reference"]["n_gpus"] == 1
    ex = f["exchange"]
    for k in ("wall_ms_per_pass", "interior_ms_per_pass", "band_ms_per_pass", "exchange_ms_per_pass",
              "exposed_exchange_ms_per_pass", "exposed_share_of_pass", "passes_timed", "halo_bytes_sent_per_pass"):
        assert k in ex, k
    assert ex["exchange_ms_per_pass"] == 30.0 / 50 and ex["exposed_exchange_ms_per_pass"] == 20.0 / 50
    assert ex["steps_per_pass"] == 2 and ex["exposed_share_of_pass"] == 0.2
    # weak scaling: no strong fields; a failed 1-GPU reference is reported, not hidden
    w = bench.scaling_fields(4, False, 2.5, phases=phases, comm_seen=4)
    assert "strong_efficiency" not in w and w["nranks_seen"] == 4
    bad = bench.scaling_fields(2, True, 2.5, t1={"error": "boom"}, comm_seen=2)
    assert bad["strong_efficiency"] is None and bad["strong_reference"] == {"error": "boom"}
    # one GPU without a communicator
    assert bench.scaling_fields(1, False, 1.0) == {"nranks_seen": 1}


def test_cpu_baseline_bounded_sample():
    """The CPU baseline stays bounded on lattices whose whole step exceeds its
    budget (C4's 8192^2 at eps 32: ~2 min per step on the GPU box's host
    share): it times the centre tile rows of one step of the same lattice and
    says so; small workloads still time whole steps.  Both carry the
    single-core serial leg."""
    big = bench.cpu_baseline(2, 512, 16, budget_s=0.05, serial_budget_s=0.05)
    assert big["value"] > 0 and "tile rows of one step" in big["sample"] and "512x512 lattice" in big["sample"]
    assert big["serial_1core"]["cores"] == 1 and big["serial_1core"]["value"] > 0
    small = bench.cpu_baseline(2, 256, 2, budget_s=2.0, serial_budget_s=0.05)
    assert small["value"] > 0 and "step(s)" in small["sample"]


def _bench(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def _error_line(stdout):
    import json
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    rec = json.loads(lines[0])
    assert "metric" in rec and "value" not in rec
    return rec


def test_error_line_single_rank_nlh_create():
    """a rank that fails prints ONE JSON line with the error,
    its rank and the stage (here nlh_create: no HIP device on this machine)
    and exits non-zero."""
    p = _bench(["--gpus", "1", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--pmc", "off"])
    assert p.returncode != 0
    rec = _error_line(p.stdout)
    assert rec["stage"] == "nlh_create" and rec["rank"] == 0 and "no HIP device" in rec["error"], rec


def test_error_line_spawned_ranks():
    """--gpus 2 without WORLD_SIZE: the launcher prints the error line of the
    first rank that failed (and nothing else on stdout)."""
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"])
    assert p.returncode != 0
    rec = _error_line(p.stdout)
    # without a GPU the first device call is rank 0's RCCL id (stage comm_id);
    # the other rank then waits in the id broadcast and is stopped
    assert rec["stage"] in ("comm_id", "nlh_create") and rec["rank"] in (0, 1) and rec["n_gpus"] == 2, rec
    assert "no HIP device" in rec["error"], rec


def test_error_line_on_hang_torchrun_form():
    """A rank that hangs in a stage (test hook NLH_BENCH_HANG_STAGE; a real
    hang would be the RCCL rendezvous or a collective) is ended by the stage
    watchdog: one error line naming the stage, exit 124.  WORLD_SIZE set, as
    torch.distributed.run launches it."""
    import json
    env = {"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
           "MASTER_PORT": str(bench.free_port()), "NLH_BENCH_STAGE_TIMEOUT": "3",
           "NLH_BENCH_HANG_STAGE": "process_group"}
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], env, timeout=120)
    assert p.returncode == 124, (p.returncode, p.stderr[-2000:])
    rec = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["stage"] == "process_group" and rec["rank"] == 0 and "did not finish" in rec["error"], rec


def test_error_line_rendezvous_timeout():
    """Rank 1 of 2 alone (its peer never starts): the gloo rendezvous blocks and
    the process-group watchdog ends it with the error line."""
    import json
    env = {"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1", "MASTER_ADDR": "127.0.0.1",
           "MASTER_PORT": str(bench.free_port()), "NLH_BENCH_STAGE_TIMEOUT": "5"}
    p = _bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--no-cpu-baseline"], env, timeout=120)
    assert p.returncode != 0
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert lines, p.stderr[-2000:]
    rec = json.loads(lines[-1])
    assert rec["rank"] == 1 and rec["stage"] == "process_group", rec


def test_read_tile_map_reference_c5():
    """--map reads the reference's partition files (C5: load_balance_25s_8n,
    5x5 tiles over 8 owners, 1-7 tiles each)."""
    path = os.path.join(ROOT, "tests", "golden", "reference_inputs", "load_balance_25s_8n.txt")
    npx, npy, own, tnx, tny = bench.read_tile_map(path)
    assert (npx, npy) == (5, 5) and own.shape == (25,) and own.min() == 0 and own.max() == 7
    counts = [int((own == o).sum()) for o in range(8)]
    assert sum(counts) == 25 and min(counts) >= 1 and max(counts) <= 7
    tok = open(path).read().split()
    assert (tnx, tny) == (int(tok[0]), int(tok[1]))
    # px outer, as the reference writes it: line i + 1 is tile (px, py) = (i // npy, i % npy)
    vals = [int(v) for v in tok[5:]]
    for i in range(25):
        px, py, o = vals[3 * i:3 * i + 3]
        assert own[px + py * npx] == o


def test_roofline_fields_two_step_pass():
    """a two-step pass must move u^t once and u^{t+2} once,
    16 B per node and launch -- 268.4 MB at C2 -- so frac = 268.4 MB / launch
    time / 8 TB/s and never exceeds 1 for a physically possible launch; the
    16-B-per-node-update figure is the separate `effective_*` key."""
    nodes = 4096 * 4096
    t = 67.60e-6  # rocprofv3 mean of k_pair_split at C2 (profiles/r05/evidence/c2)
    r = bench.roofline_fields(nodes, 2, t, 197, False)
    assert r["algorithmic_bytes_per_launch"] == 16 * nodes == 268_435_456
    assert r["node_updates_per_launch"] == 2 * nodes
    assert abs(r["achieved"] - 268_435_456 / t / 1e9) < 1e-6
    assert abs(r["frac"] - 0.4964) < 1e-3 and r["frac"] <= 1.0
    assert abs(r["effective_frac"] - 2 * r["frac"]) < 1e-12
    assert r["algorithmic_bytes_per_node_update"] == 8.0
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.HBM_PEAK_GBS
    # the bound follows the PMC limiter when there is one
    assert bench.roofline_fields(nodes, 2, t, 197, False, {"limiter": "fp64_valu_issue"})["bound"] == "fp64_valu"
    # the fastest launch HBM allows moves exactly the algorithmic bytes at peak: frac 1
    fastest = 16 * nodes / (bench.HBM_PEAK_GBS * 1e9)
    assert abs(bench.roofline_fields(nodes, 2, fastest, 197, False)["frac"] - 1.0) < 1e-12
    # test mode: the L_h[W0] plane once per pass; single-step kernels: 16 (+8) B per node-update
    rt = bench.roofline_fields(nodes, 2, t, 197, True)
    assert rt["algorithmic_bytes_per_launch"] == 24 * nodes
    r1 = bench.roofline_fields(nodes, 1, t, 197, True)
    assert r1["algorithmic_bytes_per_node_update"] == 24.0 and r1["effective_bytes_per_launch"] == 24 * nodes


def test_watchdog_quiet_stage_does_not_wake(monkeypatch):
    """The timed stage moves the watchdog's deadline without waking its
    thread (no thread start or wake-up inside the timed region), and a stage
    still expires at its deadline."""
    monkeypatch.delenv("NLH_BENCH_STAGE_TIMEOUT", raising=False)
    st = bench.Stages(0, 1)
    st.enter("warmup")
    wakes = []
    orig = st.cv.notify
    st.cv.notify = lambda *a: (wakes.append(1), orig(*a))
    st.enter("timed", quiet=True)
    assert wakes == [] and st.name == "timed"
    st.enter("report")
    assert wakes == [1]
    st.end()
    st.thread.join(5)
    assert not st.thread.is_alive()
