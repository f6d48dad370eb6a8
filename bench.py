#!/usr/bin/env python3
"""Benchmark of the explicit-Euler hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]

Workload (BASELINE.json configs[1]): a 4096 x 4096
lattice PER GPU, eps = 8, fp64, production mode (test=0: the nonlocal
operator only, as in the reference's non-test runs), synthetic test_init IC,
k = 1, dh = 1/4096, dt = eps^4 dh^2 / (8 k N(eps)).  One "step" = one explicit
Euler step of the whole lattice.

N > 1 GPUs: one process per GPU.  Under torch.distributed.run (RANK /
WORLD_SIZE set) every process is one rank; with WORLD_SIZE unset,
``--gpus N`` starts the N rank processes itself (before any GPU call) and
rank 0 prints the line.  Weak scaling by default: the lattice grows with N as
a px x py block decomposition (1x1, 2x1, 2x2, 2x4 -- the C4/C5 layouts),
ghost strips exchanged over RCCL.  ``--strong --lattice 32768`` fixes the
total lattice (C3: 2x4 blocks of 16384 x 8192 on 8 GPUs).

Prints one JSON line (rank 0) with the roofline of the dominant kernel
(HIP events on the stencil's own stream), its physical limits from rocprofv3
PMC counters of the same kernel and workload -- collected live by this run
(--pmc auto: three counter passes over tools/prof_step.py as child
processes, before this process touches the GPU), else a committed record
carrying the same library build id -- and a bounded CPU baseline (the
oracle's tiled 2d_nonlocal_async restatement on the host cores this job may
use).

Warm-up: W steps, continued (untimed) until at least --warmup-ms of stepping
has passed, so the timed region starts at the clocks a sustained run holds;
the line reports both W and the warm-up steps actually run.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import tempfile
import threading
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

EPS = 8
NB = 4096                      # lattice per GPU (each direction)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_VEC_PEAK_TFLOPS = 78.6    # 256 CU x 64 lanes x 2 x 2.4 GHz (spec)
FP64_LANE_OPS_PEAK = 256 * 64 * 2.4e9  # f64 VALU lane-operations per second (spec clock)
BYTES_PER_NODE = 16.0          # read u once + write u' once


def read_tile_map(path):
    """The reference's partition file (src/2d_nonlocal_distributed.cpp:476-484):
    line 1 "nx ny npx npy dh" (tile size, tile counts, spacing), then npx*npy
    lines "px py owner".  Returns (npx, npy, owner[px + py*npx], tile nx, tile ny)."""
    import numpy as np
    tok = open(path).read().split()
    tnx, tny, npx, npy = (int(v) for v in tok[:4])
    own = np.full(npx * npy, -1, dtype=np.int32)
    vals = [int(v) for v in tok[5:5 + 3 * npx * npy]]
    for i in range(0, len(vals), 3):
        px, py, o = vals[i:i + 3]
        own[px + py * npx] = o
    if (own < 0).any():
        raise ValueError(f"{path}: not every tile has an owner")
    return npx, npy, own, tnx, tny


def decomposition(n: int):
    """px x py blocks for n ranks: 1x1, 2x1, 2x2, 2x4,
    else px the largest power of two with px^2 <= n dividing n."""
    if n == 2:
        return 2, 1
    px = 1
    while (2 * px) * (2 * px) <= n and n % (2 * px) == 0:
        px *= 2
    return px, n // px


def progress(msg: str) -> None:
    """A progress line on stderr (stdout carries only the JSON line): a long
    bench (live PMC passes, the CPU baseline) keeps writing while it runs."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def host_cpu_share() -> int:
    """Host threads this job may use: the CPU affinity mask, capped by the
    cgroup CPU quota and by OMP_NUM_THREADS when the launcher sets it (the GPU
    box exports its per-GPU CPU share there; nproc shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, math.ceil(int(quota) / int(period))))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(nthreads: int, nb: int = NB, eps: int = EPS, test: bool = False,
                 budget_s: float = 15.0, serial_budget_s: float = 8.0) -> dict:
    """Oracle restatement of 2d_nonlocal_async (np x np tiles, one task per
    tile per step, a barrier per step) on the same nb^2 / eps workload,
    bounded to ~budget_s of wall time, plus the single-core serial restatement
    of 2d_nonlocal_serial on a lattice sized to
    ~serial_budget_s."""
    import nonlocalheatequation_amd as N
    from oracle import oracle as O  # test infrastructure: baseline leg only

    dh = 1.0 / nb
    dt = eps ** 4 * dh * dh / (8.0 * N.disk_count(eps))
    p = O.params(nb, nb, eps, 1.0, dt, dh, int(test))
    u = O.test_init(p)
    tiles = max(1, nb // 128)  # 128 x 128-node tiles
    th = -(-nb // tiles)
    # probe: one tile row from the middle of the lattice -> the cost of a whole step
    mid = (tiles // 2) * tiles
    tp = O.time_tiles(p, 0, tiles, tiles, mid, tiles, u, nthreads)
    if tp * tiles <= budget_s:
        t1 = O.run_tiled(p, 1, tiles, tiles, u, nthreads)
        if t1 > budget_s / 3:  # one step fills the budget: it is the sample
            steps, t = 1, t1
        else:
            steps = int(max(1, min(200, budget_s / max(t1, 1e-3) - 1)))
            t = O.run_tiled(p, steps, tiles, tiles, u, nthreads)
        rate = nb * nb * steps / t / 1e9
        what = (f"{steps} step(s) ({t:.1f} s{'' if steps == 1 and t == t1 else ', after 1 warm-up step'})")
    else:
        # a whole step would take ~tp * tiles s (C4's 8192^2 at eps 32: ~2 min):
        # time the centre tile rows of one step of the same lattice, as many as
        # fill the budget
        rows = int(min(tiles, max(1, budget_s / tp)))
        first = ((tiles - rows) // 2) * tiles
        t = O.time_tiles(p, 0, tiles, tiles, first, rows * tiles, u, nthreads)
        steps = 1
        rate = rows * th * nb / t / 1e9
        what = (f"the centre {rows} of its {tiles} tile rows of one step ({t:.1f} s; a whole step "
                f"~{tp * tiles:.0f} s)")
    # single core: a square lattice of the same eps / mode sized from the
    # tiled per-thread rate, one step of the serial restatement
    per_thread = rate * 1e9 / max(1, nthreads)
    side = int(min(nb, max(64, math.sqrt(serial_budget_s * per_thread)))) // 64 * 64
    ps = O.params(side, side, eps, 1.0, eps ** 4 / (8.0 * side * side * N.disk_count(eps)), 1.0 / side, int(test))
    us = O.test_init(ps)
    t0 = time.perf_counter()
    O.run(ps, 1, us, nthreads=1)
    ts = time.perf_counter() - t0
    serial = {"value": side * side / ts / 1e9, "unit": "Gnode-updates/s", "cores": 1,
              "sample": f"{side}x{side} lattice, eps={eps}, test={int(test)}, 1 step ({ts:.1f} s), "
                        f"oracle/nlh_oracle.c nlh_oracle_run on one thread (2d_nonlocal_serial restatement)"}
    return {"value": rate, "unit": "Gnode-updates/s", "cores": nthreads, "kind": "port",
            "host_cpus_visible": os.cpu_count(),
            "sample": f"{nb}x{nb} lattice, eps={eps}, test={int(test)}, {what}, "
                      f"{tiles}x{tiles} tiles on {nthreads} threads (the job's host CPU share), "
                      f"oracle/nlh_oracle.c run_tiled (-O3 -ffp-contract=off)",
            "serial_1core": serial}


def workload_key(nb, eps, strong, test) -> str:
    return f"{'strong' if strong else 'weak'}_{nb}_eps{eps}_{'test' if test else 'prod'}"


def workload_name(nb, eps, strong, test, nx, ny) -> str:
    mode = "test mode (manufactured source)" if test else "production step (test=0)"
    if not strong and nb == NB and eps == EPS:
        return f"C2: {nb}x{nb} lattice per GPU, eps={eps}, {mode}"
    if strong:
        return f"{nx}x{ny} lattice in total (strong scaling), eps={eps}, {mode}"
    return f"{nb}x{nb} lattice per GPU, eps={eps}, {mode}"


def read_pmc(kernel_name: str, wkey: str, build_id: str):
    """The committed rocprofv3 PMC summary of this kernel on this workload
    (tools/pmc_summary.py: FETCH_SIZE doubled per the gfx950 correction +
    WRITE_SIZE, SQ_INSTS_VALU; separate passes), if one exists AND was
    profiled on a library with this build id."""
    path = os.path.join(ROOT, "profiles", "pmc", f"{kernel_name}__{wkey}.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, path
    if d.get("kernel_match") != kernel_name or d.get("workload") != wkey or d.get("build_id") != build_id:
        return None, path
    return d, path


# one counter group per rocprofv3 pass (MI355X_MICROARCH.md: FETCH_SIZE and
# WRITE_SIZE cannot share a pass; <= 8 SQ counters per pass)
PMC_PASSES = ["FETCH_SIZE", "WRITE_SIZE",
              "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"]


def live_pmc(args, wkey: str):
    """rocprofv3 --pmc passes over tools/prof_step.py running this bench's
    workload, each a child process under its own time limit.  Called before
    this process loads libnlh or touches the GPU.  Returns the record
    read_pmc would return (same keys; kernel, node-updates per launch and
    build id as the profiled program reported them), or None when rocprofv3
    is unavailable or a pass fails."""
    import csv
    import shutil
    import statistics
    import tempfile
    prof = shutil.which("rocprofv3")
    if not prof:
        return None
    env = dict(os.environ, NLH_N=str(args.lattice), NLH_EPS=str(args.eps), NLH_TEST=str(int(args.test_mode)),
               NLH_KERNEL=args.kernel, NLH_INFLUENCE=args.influence, NLH_SEG=str(args.seg_rows),
               TMPDIR="/tmp")
    vals, durs, seen = {}, {}, set()
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        for i, grp in enumerate(PMC_PASSES):
            progress(f"live PMC pass {i + 1}/{len(PMC_PASSES)}: {grp}")
            out = os.path.join(td, f"p{i}")
            cmd = ["timeout", "-s", "KILL", "120", prof, "--pmc", *grp.split(), "--kernel-trace",
                   "--output-format", "csv", "-d", out, "-o", "run", "--",
                   sys.executable, os.path.join(ROOT, "tools", "prof_step.py")]
            try:
                r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True,
                                   timeout=150)
            except (OSError, subprocess.SubprocessError):
                return None
            ok = [l.split() for l in r.stdout.splitlines() if l.startswith("ok ")]
            if r.returncode != 0 or not ok or len(ok[-1]) != 5:
                return None
            seen.add(tuple(ok[-1][1:]))
            kernel_name, spp, nodes, build_id = ok[-1][1], int(ok[-1][2]), int(ok[-1][3]), ok[-1][4]
            key = kernel_name + "<"
            for root, _, files in os.walk(out):
                for fn in files:
                    path = os.path.join(root, fn)
                    if fn.endswith("counter_collection.csv"):
                        for row in csv.DictReader(open(path)):
                            if key in row["Kernel_Name"]:
                                vals.setdefault(row["Counter_Name"], {}).setdefault(
                                    row["Kernel_Name"], []).append(float(row["Counter_Value"]))
                    elif fn.endswith("kernel_trace.csv"):
                        for row in csv.DictReader(open(path)):
                            if key in row["Kernel_Name"]:
                                durs.setdefault(row["Kernel_Name"], []).append(
                                    int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    # per pass: the median of each kernel instance, summed over the instances a
    # pass launches (one for every kernel libnlh has today)
    med = {c: sum(statistics.median(v) for v in per.values()) for c, per in vals.items()}
    durs = [sum(statistics.median(v) for v in durs.values())] if durs else []
    if len(seen) != 1 or not {"FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU"} <= set(med):
        return None
    node_updates = nodes * spp
    rd, wr = 2.0 * med["FETCH_SIZE"] * 1024, med["WRITE_SIZE"] * 1024  # gfx950 FETCH_SIZE half-count
    rec = {"kernel_match": kernel_name, "workload": wkey, "build_id": build_id, "source": "live",
           "median": med, "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
           "hbm_bytes_per_launch": rd + wr, "valu_insts_per_launch": med["SQ_INSTS_VALU"],
           "node_updates_per_launch": node_updates,
           "profiled_duration_us_median": statistics.median(durs) / 1e3 if durs else None,
           "correction": "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads), KiB -> bytes"}
    if med.get("SQ_WAVE_CYCLES"):
        rec["share_of_wave_cycles"] = {k: med[k] / med["SQ_WAVE_CYCLES"] for k in ("SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU")
                                       if k in med}
    return rec


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_ranks(n: int) -> int:
    """Start n rank processes of this script (RANK / LOCAL_RANK / WORLD_SIZE /
    MASTER_* in their environment) and wait for them.  The parent never
    touches the GPU."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        outs = tempfile.TemporaryFile(mode="w+")
        procs.append((subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                       stdout=outs), outs, r))
    # a rank that fails would leave the others blocked in a collective: stop
    # them (these exact child processes) as soon as one exits non-zero; the
    # first rank to fail is the one whose error line this launcher prints
    rc = 0
    first_bad = None
    live = [p for p, _, _ in procs]
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0:
                rc = max(rc, abs(r))
                if first_bad is None:
                    first_bad = p
                for q in live:
                    q.terminate()
        time.sleep(0.2)
    lines = {}
    for p, f, r in procs:
        f.seek(0)
        lines[r] = [l for l in f.read().splitlines() if l.startswith("{")]
        f.close()
    if rc == 0:
        for l in lines.get(0, []):
            print(l, flush=True)
        return 0
    bad_rank = next(r for p, _, r in procs if p is first_bad)
    errs = [l for l in lines.get(bad_rank, []) if '"error"' in l]
    if errs:
        print(errs[-1], flush=True)
    else:
        code = next(p.returncode for p, _, r in procs if r == bad_rank)
        print(json.dumps({"error": f"rank {bad_rank} exited with code {code} without an error line",
                          "rank": bad_rank, "stage": "unknown", "n_gpus": n}), flush=True)
    return rc


class stdout_to_stderr:
    """RCCL prints its version banner on stdout when a communicator starts:
    keep fd 1 for the one JSON line (the banner goes to stderr)."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


class Stages:
    """Where a rank is, for the one error line a failed or hung run prints
    (the first real multi-GPU run must be diagnosable).

    One watchdog thread, started with the object, sleeps until the current
    stage's deadline; enter(name) moves the deadline (NLH_BENCH_STAGE_TIMEOUT
    seconds overrides every limit).  If a stage has not ended by its deadline
    the rank prints {"error", "rank", "stage", ...} on stdout and exits 124 --
    ctypes calls release the GIL, so the watchdog runs while the main thread
    sits in nlh_create / RCCL init / a collective.  enter(name, quiet=True)
    (the timed stage) only moves the deadline further out without waking the
    watchdog, so no thread starts or wakes inside the timed region (VERDICT r5:
    round 5 started a threading.Timer right before t0).  fail() prints the
    same line for an exception or a failed check."""
    LIMITS = {"process_group": 300, "comm_id": 300, "nlh_create": 900, "comm_check": 300,
              "first_exchange": 300, "warmup": 900, "timed": 3600, "report": 3600}

    def __init__(self, rank: int, nranks: int):
        self.rank, self.nranks, self.name, self.t0 = rank, nranks, "start", time.time()
        self.cv = threading.Condition()
        self.deadline = None  # time.monotonic() at which the current stage expires
        self.limit = 0.0
        self.done = False
        self.thread = threading.Thread(target=self._watch, name="bench-watchdog", daemon=True)
        self.thread.start()

    def line(self, error: str, stage=None) -> str:
        return json.dumps({"error": error, "rank": self.rank, "stage": stage or self.name,
                           "n_gpus": self.nranks, "metric": "Gnode-updates/s (nodes*steps/s) fp64",
                           "elapsed_s": round(time.time() - self.t0, 3)})

    def _watch(self) -> None:
        with self.cv:
            while not self.done:
                if self.deadline is None:
                    self.cv.wait()
                    continue
                left = self.deadline - time.monotonic()
                if left > 0:
                    self.cv.wait(left)
                    continue
                self.done = True
                name, limit = self.name, self.limit
                break
            else:
                return
        sys.stderr.flush()
        os.write(1, (self.line(f"stage '{name}' did not finish within {limit:g} s (hung: a peer rank, the RCCL "
                               f"rendezvous or a collective)", name) + "\n").encode())
        os._exit(124)

    def enter(self, name: str, quiet: bool = False) -> None:
        env = os.environ.get("NLH_BENCH_STAGE_TIMEOUT")
        limit = float(env) if env else float(self.LIMITS.get(name, 3600))
        with self.cv:
            deadline = time.monotonic() + limit
            # quiet: the watchdog's current wait ends no later than the new
            # deadline, so it need not wake now (it re-reads the deadline then)
            quiet = quiet and self.deadline is not None and deadline >= self.deadline
            self.name, self.limit, self.deadline = name, limit, deadline
            if not quiet:
                self.cv.notify()
        if os.environ.get("NLH_BENCH_HANG_STAGE") == name:  # test hook: tests/test_bench.py
            time.sleep(1e6)

    def end(self) -> None:
        with self.cv:
            self.done = True
            self.cv.notify()

    def fail(self, error: str, code: int) -> int:
        self.end()
        print(self.line(error), flush=True)
        print(f"rank {self.rank}: {self.name}: {error}", file=sys.stderr, flush=True)
        return code


def roofline_fields(local_nodes: int, steps_per_pass: int, avg_launch_s: float, disk_points: int,
                    test_lw: bool, physical=None) -> dict:
    """roofline of the dominant kernel.

    achieved = the ALGORITHMIC bytes one launch must move / its average
    duration.  A launch (pass) advances steps_per_pass time steps of
    local_nodes nodes and must read u^t once and write u^{t+steps_per_pass}
    once -- 16 B per node and pass, plus 8 B per node when the fast test mode
    reads its L_h[W0] plane (once per pass) -- so a two-step pass moves 8 B per
    node-update and its frac is a true fraction of HBM bandwidth (<= 1).  The
    16-B-per-node-update figure of SURVEY 8(d), which charges every time step
    a full read and write, is kept as the `effective_*` keys.  bound: the
    ceiling the PMC counters name (physical.limiter), "hbm" without them."""
    bytes_node_pass = BYTES_PER_NODE + (8.0 if test_lw else 0.0)
    alg_bytes = bytes_node_pass * local_nodes
    nu_launch = local_nodes * steps_per_pass
    achieved = alg_bytes / avg_launch_s / 1e9
    eff_bytes = (BYTES_PER_NODE + (8.0 / steps_per_pass if test_lw else 0.0)) * nu_launch
    eff = eff_bytes / avg_launch_s / 1e9
    fp64_equiv = 2.0 * disk_points * nu_launch / avg_launch_s / 1e12
    limiter = (physical or {}).get("limiter")
    bound = "hbm" if limiter in (None, "hbm") else "fp64_valu"
    return {
        "bound": bound,
        "bound_source": "physical.limiter (PMC)" if limiter else "algorithmic (no PMC record)",
        "achieved": achieved,
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "achieved_is": ("algorithmic bytes one launch must move (u^t read once, u^{t+%d} written once%s) / its "
                        "average duration" % (steps_per_pass, ", L_h[W0] read once" if test_lw else "")),
        "algorithmic_bytes_per_launch": alg_bytes,
        "algorithmic_bytes_per_node_update": alg_bytes / nu_launch,
        "node_updates_per_launch": nu_launch,
        "effective_bytes_per_launch": eff_bytes,
        "effective_gbs": eff,
        "effective_frac": eff / HBM_PEAK_GBS,
        "effective_is": "16 B per node-update (SURVEY 8(d): every step reads u and writes u') / launch time",
        "fp64_direct_sum_equiv_tflops": fp64_equiv,
        "fp64_direct_sum_equiv_frac": fp64_equiv / FP64_VEC_PEAK_TFLOPS,
    }


def strong_reference(args) -> dict:
    """T1 of the strong-scaling efficiency T1 / (N T_N): this bench on ONE GPU
    over the same total lattice, run as a child process before this rank
    touches the GPU (the other ranks wait in the rendezvous meanwhile)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "ROLE_RANK",
                        "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    cmd = [sys.executable, os.path.abspath(__file__), "--gpus", "1", "--strong", "--lattice", str(args.lattice),
           "--eps", str(args.eps), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--kernel", args.kernel, "--influence", args.influence, "--pmc", "off", "--no-cpu-baseline"]
    if args.test_mode:
        cmd.append("--test-mode")
    progress("strong scaling: the 1-GPU reference run of the same lattice")
    try:
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=900)
    except (OSError, subprocess.SubprocessError) as e:
        return {"error": f"1-GPU reference run failed: {e}"}
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    if r.returncode != 0 or not lines:
        return {"error": f"1-GPU reference run exited {r.returncode}: {r.stderr[-400:]}"}
    one = json.loads(lines[-1])
    return {"ms_per_step": one["ms_per_step"], "value": one["value"], "build_id": one.get("build_id"),
            "kernel_avg_us": one["roofline"]["kernel_avg_us"]}


def scaling_fields(nranks: int, strong: bool, ms_per_step: float, t1=None, phases=None,
                   comm_seen=None) -> dict:
    """The N > 1 fields of the bench line (tests/test_bench.py checks the
    schema on CPU):
      nranks_seen        ranks of the RCCL communicator as RCCL reports them
                         (ncclCommCount, identical on every rank; 1 without one)
      exchange           per-pass phase times (nlh_phase_time, max over ranks):
                         interior / band / exchange kernels, wall, and the
                         exposed exchange = wall - interior
      strong_efficiency  T1 / (N T_N), T1 from the 1-GPU run of the same lattice
    """
    out = {"nranks_seen": comm_seen if comm_seen else 1}
    if phases:
        P = max(1, phases["passes"])
        per = {k: phases[k] / P for k in ("wall_ms", "interior_ms", "band_ms", "exchange_ms", "exposed_exchange_ms")}
        out["exchange"] = {
            "passes_timed": phases["passes"], "steps_per_pass": phases["steps"] / P,
            "wall_ms_per_pass": per["wall_ms"], "interior_ms_per_pass": per["interior_ms"],
            "band_ms_per_pass": per["band_ms"], "exchange_ms_per_pass": per["exchange_ms"],
            "exposed_exchange_ms_per_pass": per["exposed_exchange_ms"],
            "exposed_share_of_pass": per["exposed_exchange_ms"] / per["wall_ms"] if per["wall_ms"] > 0 else None,
            "halo_bytes_sent_per_pass": phases.get("halo_bytes_sent"),
            "over_ranks": "max",
            "source": "nlh_phase_time: HIP event pairs on the streams the interior, edge-band and exchange "
                      "(pack, grouped ncclSend/ncclRecv, unpack) run on, a separate untimed run after the "
                      "timed region",
        }
    if strong and nranks > 1:
        if t1 and "ms_per_step" in t1:
            out["strong_efficiency"] = t1["ms_per_step"] / (nranks * ms_per_step)
            out["strong_reference"] = dict(t1, n_gpus=1)
        else:
            out["strong_efficiency"] = None
            out["strong_reference"] = t1
    return out


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--kernel", default="fast", choices=["fast", "exact", "auto"])
    ap.add_argument("--seg-rows", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--warmup-ms", type=float, default=300.0,
                    help="continue the untimed warm-up until this much stepping has passed")
    ap.add_argument("--pmc", default="auto", choices=["auto", "off"],
                    help="auto: collect the roofline's PMC counters live (N=1, rocprofv3 on PATH)")
    ap.add_argument("--phase-passes", type=int, default=50,
                    help="passes of the untimed phase-timing run (exchange report; runs with several owners)")
    # secondary workloads (the default line is C2): --eps 32 --lattice 8192 is
    # C4; --lattice 32768 --strong is C3 (total lattice fixed as N grows);
    # --test-mode times the manufactured-solution step and reports its L2
    ap.add_argument("--eps", type=int, default=EPS)
    ap.add_argument("--lattice", type=int, default=NB, help="lattice edge per GPU (weak) or total (--strong)")
    ap.add_argument("--strong", action="store_true")
    ap.add_argument("--blocks", default="",
                    help="PXxPY block grid instead of the per-N default (one GPU under NLH_VIRTUAL_RANKS: "
                         "e.g. --strong --lattice 32768 --blocks 2x4 runs C3's 8 ranks on one device)")
    ap.add_argument("--test-mode", action="store_true")
    # uneven ownership (C5): the reference's --file tile map, tiles resized to
    # --tile (one GPU runs the owners as NLH_VIRTUAL_RANKS; N > 1 needs one
    # rank per owner); no CPU baseline / live PMC for this layout
    ap.add_argument("--map", default="", help="tile -> owner map in the reference's --file format")
    ap.add_argument("--tile", type=int, default=0, help="tile edge for --map (default: the file's)")
    # J(r) = 1 - r (problem_description.tex:159; not the BASELINE metric, whose J = 1)
    ap.add_argument("--influence", default="constant", choices=["constant", "linear"])
    args = ap.parse_args()
    eps, nb = args.eps, args.lattice

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        print(f"--gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        return 2
    nranks = world
    st = Stages(rank, nranks)
    try:
        return _run(args, st, rank, local, nranks)
    except Exception as e:  # noqa: BLE001 -- every failure ends in the one error line
        return st.fail(f"{type(e).__name__}: {e}", 1)


def _run(args, st: Stages, rank: int, local: int, nranks: int) -> int:
    eps, nb = args.eps, args.lattice
    # strong scaling: the 1-GPU time of the same lattice, before any GPU call here
    t1 = strong_reference(args) if args.strong and nranks > 1 and rank == 0 else None

    wkey = workload_key(nb, eps, args.strong, args.test_mode) + ("_linear" if args.influence == "linear" else "")
    pmc_live = None
    if args.pmc == "auto" and args.gpus == 1 and "WORLD_SIZE" not in os.environ and not args.map:
        pmc_live = live_pmc(args, wkey)  # child processes; this one has not loaded libnlh yet

    import nonlocalheatequation_amd as N
    build_id = N.build_id()
    if build_id != N.source_build_id():
        return st.fail(f"libnlh build {build_id} does not match the sources ({N.source_build_id()}): make lib", 4)

    dist = None
    if nranks > 1:
        st.enter("process_group")
        import torch.distributed as dist  # control plane only (id broadcast, barrier, max)
        dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            return st.fail(f"process group has {dist.get_world_size()} ranks, expected {args.gpus}", 3)

    px, py = decomposition(nranks)
    own = None
    if args.map:
        px, py, own, tnx, tny = read_tile_map(args.map)
        if args.tile:
            tnx = tny = args.tile
        nowners = int(own.max()) + 1
        if nranks > 1 and nowners != nranks:
            return st.fail(f"--map {args.map} has {nowners} owners, the job {nranks} ranks", 2)
    elif args.blocks:
        px, py = (int(v) for v in args.blocks.lower().split("x"))
        if nranks > 1 and px * py != nranks:
            return st.fail(f"--blocks {args.blocks} needs one block per rank", 2)
    if own is not None:
        nx, ny = tnx * px, tny * py
        nb = nx
    elif args.strong:
        if nb % px or nb % py:
            return st.fail(f"--lattice {nb} is not divisible by the {px}x{py} block grid", 2)
        nx, ny = nb, nb
    else:
        nx, ny = nb * px, nb * py
    dh = 1.0 / nb
    dt = eps ** 4 * dh * dh / (8.0 * N.disk_count(eps))
    if args.influence == "linear":
        dt /= 5.0  # c = 40 k / (eps dh)^4: five times J = 1's c, same stability margin

    comm_id = None
    if nranks > 1:
        st.enter("comm_id")
        obj = [N.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]

    st.enter("nlh_create")  # device, blocks and (N > 1) the RCCL communicator init
    with stdout_to_stderr():
        s = N.Solver(nx, ny, eps, 1.0, dt, dh, test=args.test_mode, kernel=args.kernel, device=local,
                     rank=rank, nranks=nranks, tiles=(px, py), owner=own, comm_id=comm_id,
                     seg_rows=args.seg_rows, influence=args.influence)
    info = s.info()
    # every rank owns exactly one block of the px x py grid, and the RCCL
    # communicator itself (ncclCommCount / ncclCommUserRank, nlh_info) must
    # see all N ranks, each once -- else the line would claim GPUs that did not
    # take part
    comm_seen = None
    if dist is not None:
        st.enter("comm_check")
        lst = [None] * nranks
        dist.all_gather_object(lst, (info.owned_nodes, info.nblocks, info.comm_nranks, info.comm_rank))
        owned = [o[0] for o in lst]
        if sum(owned) != nx * ny or any(o == 0 for o in owned):
            return st.fail(f"ranks own {owned} nodes of {nx * ny}", 3)
        counts = {o[2] for o in lst}
        ranks_seen = sorted(o[3] for o in lst)
        if counts != {nranks} or ranks_seen != list(range(nranks)):
            return st.fail(f"RCCL communicator sizes {sorted(counts)} / ranks {ranks_seen}, expected {nranks} "
                           f"ranks", 5)
        comm_seen = nranks
    s.test_init()
    # the first pass(es): the first ghost exchange over RCCL on N > 1
    st.enter("first_exchange")
    s.run(max(1, info.steps_per_pass))
    s.synchronize()
    if dist is not None:
        dist.barrier()
    # warm-up: W steps, then more until --warmup-ms of stepping has passed (the
    # clocks a sustained run holds); every rank runs the same count (rank 0's)
    st.enter("warmup")
    s.run(args.warmup)
    s.synchronize()
    warm = args.warmup + max(1, info.steps_per_pass)
    tw = time.perf_counter()
    chunk = max(2, args.warmup)
    while warm < 100000:
        go = (time.perf_counter() - tw) * 1e3 < args.warmup_ms
        if dist is not None:  # rank 0 decides, so every rank runs the same passes (the exchange is collective)
            import torch
            g = torch.tensor([int(go)], dtype=torch.int64)
            dist.broadcast(g, src=0)
            go = bool(g.item())
        if not go:
            break
        s.run(chunk)
        s.synchronize()
        warm += chunk

    def barrier():
        s.synchronize()
        if dist is not None:
            dist.barrier()

    # the measurement path itself warmed up: two untimed runs of exactly the
    # timed sequence (event pair, K steps, polling wait, readback).  The first
    # timed runs of a process start their first launch 6-9 us later than the
    # rest (r06, tools/host_gap.py: host-side first-use costs), and with
    # NLH_GRAPH the graphs of these K steps are captured here, not in the
    # timed region.  They count as warm-up steps.
    for _ in range(2):
        barrier()
        s.kernel_timing(True)
        s.run(args.steps)
        s.synchronize()
        s.kernel_time()
        s.host_time()
        s.kernel_timing(False)
        warm += args.steps

    barrier()
    if rank == 0:
        progress(f"warm-up done ({warm} steps); timing {args.steps} steps")
    # HIP events on the stencil stream bracket the timed region (one pair);
    # the average launch duration below is their span / launches
    s.kernel_timing(True)
    st.enter("timed", quiet=True)  # no watchdog wake-up inside the timed region
    t0 = time.perf_counter()
    s.run(args.steps)
    t_enq = time.perf_counter()
    s.synchronize()
    t1_wall = time.perf_counter()
    k_ms, k_n = s.kernel_time()
    lib_host = s.host_time()
    s.kernel_timing(False)
    barrier()
    elapsed = t1_wall - t0
    # where the timed region went: t0 -> run() returned,
    # -> synchronize() returned, and the stream-event span of the passes
    host = {"wall_us": elapsed * 1e6, "enqueue_us": (t_enq - t0) * 1e6, "sync_us": (t1_wall - t_enq) * 1e6,
            "event_span_us": k_ms * 1e3, "outside_events_us": elapsed * 1e6 - k_ms * 1e3,
            "lib": {k: v for k, v in lib_host.items() if k != "event_span_us"},
            "note": "outside_events_us = wall - event span: the first launch reaching the GPU plus the host "
                    "seeing the last one finish (lib.end_seen_us / sync_return_us: from nlh_run's entry)"}
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    st.enter("report")
    l2 = s.compute_l2(s.step_index) if args.test_mode else None  # after the timed region

    # exchange report (several owners): a separate, untimed run with an event
    # pair around every pass's interior, bands and exchange
    phases = None
    if (nranks > 1 or info.owners > 1) and args.phase_passes > 0:
        barrier()
        s.kernel_timing(3)
        s.run(args.phase_passes * info.steps_per_pass)
        s.synchronize()
        ph = s.phase_time()
        s.kernel_timing(False)
        vals = [ph.wall_ms, ph.interior_ms, ph.band_ms, ph.exchange_ms, ph.exposed_exchange_ms]
        if dist is not None:
            import torch
            tv = torch.tensor(vals, dtype=torch.float64)
            dist.all_reduce(tv, op=dist.ReduceOp.MAX)
            vals = tv.tolist()
        phases = dict(zip(("wall_ms", "interior_ms", "band_ms", "exchange_ms", "exposed_exchange_ms"), vals),
                      passes=ph.passes, steps=ph.steps, halo_bytes_sent=info.halo_bytes_sent)
        barrier()

    total_nodes = nx * ny
    value = total_nodes * args.steps / elapsed / 1e9
    ms_per_step = elapsed * 1e3 / args.steps
    local_nodes = info.owned_nodes
    # one stencil launch (a "pass") advances steps_per_pass time steps: 2 for
    # the temporally blocked production kernel k_pair_split, 1 for k_fast / k_exact
    spp = info.steps_per_pass
    kname = info.pass_kernel
    passes = max(k_n // spp, 1)
    avg_launch_s = (k_ms / 1e3) / passes
    nu_launch = local_nodes * spp
    test_lw = bool(args.test_mode and info.kernel == N.KERNEL_FAST)
    pmc, pmc_path = None, None
    if pmc_live and pmc_live["kernel_match"] == kname and pmc_live["build_id"] == build_id \
            and pmc_live["node_updates_per_launch"] == nu_launch:
        pmc, pmc_path = pmc_live, "live"
    elif nranks == 1:
        pmc, pmc_path = read_pmc(kname, wkey, build_id)
    traffic = pmc["hbm_bytes_per_launch"] if pmc else None
    physical = None
    if pmc:
        # what the kernel actually moves and issues (PMC), and the ceiling
        # those counts allow: min(HBM spec / bytes, f64 VALU issue / lane-ops)
        b_nu = pmc["hbm_bytes_per_launch"] / pmc["node_updates_per_launch"]
        ops_nu = pmc["valu_insts_per_launch"] * 64.0 / pmc["node_updates_per_launch"]
        hbm_ceiling = HBM_PEAK_GBS * 1e9 / b_nu / 1e9
        valu_ceiling = FP64_LANE_OPS_PEAK / ops_nu / 1e9
        rate_launch = nu_launch / avg_launch_s / 1e9  # G node-updates/s of the kernel alone
        physical = {
            "hbm_bytes_per_node_update": b_nu,
            "hbm_frac": pmc["hbm_bytes_per_launch"] / avg_launch_s / 1e9 / HBM_PEAK_GBS,
            "valu_lane_ops_per_node_update": ops_nu,
            "valu_frac": pmc["valu_insts_per_launch"] * 64.0 / avg_launch_s / FP64_LANE_OPS_PEAK,
            "hbm_ceiling_gnu": hbm_ceiling,
            "valu_ceiling_gnu": valu_ceiling,
            "ceiling_gnu": min(hbm_ceiling, valu_ceiling),
            "limiter": "hbm" if hbm_ceiling < valu_ceiling else "fp64_valu_issue",
            "kernel_rate_gnu": rate_launch,
            "frac_of_ceiling": rate_launch / min(hbm_ceiling, valu_ceiling),
            "wait_share_of_wave_cycles": pmc.get("share_of_wave_cycles", {}).get("SQ_WAIT_ANY"),
            "source": "live rocprofv3 --pmc passes of this run (tools/prof_step.py, same workload)"
                      if pmc_path == "live" else os.path.relpath(pmc_path, ROOT),
            "build_id": pmc.get("build_id"),
        }

    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and nranks == 1 and args.influence == "constant" and own is None:
            # bounded sample on the workload's own lattice (one step when that
            # fills the budget: C4) and a single-core serial leg
            progress("CPU baseline (bounded sample, after the timed region)")
            cpu = cpu_baseline(host_cpu_share(), nb, eps, args.test_mode)
        result = {
            "metric": f"Gnode-updates/s (nodes*steps/s) eps={eps} fp64",
            "value": value,
            "unit": "Gnode-updates/s",
            "n_gpus": nranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "warmup_steps_run": warm,
            "build_id": build_id,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if args.strong or own is not None else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (test_init IC sin(2 pi x) sin(2 pi y); no dataset)",
            "config": {
                "workload": workload_name(nb, eps, args.strong or own is not None, args.test_mode, nx, ny)
                            + f", {args.kernel} kernel"
                            + (", J(r) = 1 - r" if args.influence == "linear" else "")
                            + (f", {px}x{py} blocks + RCCL ghost exchange" if nranks > 1 and own is None else "")
                            + (f", tile map {os.path.basename(args.map)}: {px}x{py} tiles of {tnx}x{tny}, "
                               f"{int(own.max()) + 1} owners, RCCL ghost exchange" if own is not None else ""),
                "lattice": [nx, ny], "eps": eps, "blocks": [px, py], "test_mode": args.test_mode,
                "disk_points": info.disk_points, "dt": dt, "dh": dh, "kernel": args.kernel,
                "parallelism": f"{px}x{py} block decomposition, one rank per GPU" if nranks > 1 else "1 GPU",
                "virtual_ranks": info.owners if nranks == 1 and info.owners > 1 else None,
                **({"tile_map": os.path.basename(args.map), "tile": [tnx, tny],
                    "tiles_per_owner": [int(c) for c in __import__("numpy").bincount(own)]}
                   if own is not None else {}),
            },
            "roofline": dict(roofline_fields(local_nodes, spp, avg_launch_s, info.disk_points, test_lw, physical),
                             traffic=traffic, kernel=kname, steps_per_launch=spp,
                             kernel_avg_us=avg_launch_s * 1e6, kernel_launches_timed=passes, physical=physical),
            "host": host,
            "cpu_baseline": cpu,
        }
        result.update(scaling_fields(nranks, args.strong, ms_per_step, t1, phases, comm_seen))
        if l2 is not None:
            result["config"]["l2_error"] = l2  # reference error_l2 at the final step
        print(json.dumps(result), flush=True)
    s.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    st.end()
    return 0


if __name__ == "__main__":
    sys.exit(main())
