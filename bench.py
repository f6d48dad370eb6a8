#!/usr/bin/env python3
"""Benchmark of the explicit-Euler hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]

Workload (BASELINE.json configs[1]): a 4096 x 4096
lattice PER GPU, eps = 8, fp64, production mode (test=0: the nonlocal
operator only, as in the reference's non-test runs), synthetic test_init IC,
k = 1, dh = 1/4096, dt = eps^4 dh^2 / (8 k N(eps)).  One "step" = one explicit
Euler step of the whole lattice.  N > 1 GPUs: one process per GPU (launched by
torch.distributed.run), the lattice grows with N (weak scaling) as a px x py
block decomposition with eps-wide ghost strips exchanged over RCCL each step.

Prints one JSON line (rank 0) with the roofline of the dominant kernel
(HIP events on the stencil's own stream) and a bounded CPU baseline (the
oracle's tiled 2d_nonlocal_async restatement on the host cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import nonlocalheatequation_amd as N  # noqa: E402

EPS = 8
NB = 4096                      # lattice per GPU (each direction)
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_VEC_PEAK_TFLOPS = 78.6    # 256 CU x 64 lanes x 2 x 2.4 GHz (spec)
BYTES_PER_NODE = 16.0          # read u once + write u' once


def decomposition(n: int):
    px = 1
    while px * px < n:
        px *= 2
    while n % px:
        px //= 2
    return px, n // px


def cpu_baseline(nthreads: int, nb: int = NB, eps: int = EPS, test: bool = False,
                 budget_s: float = 12.0) -> dict:
    """Oracle restatement of 2d_nonlocal_async (np x np tiles, one task per
    tile per step, a barrier per step) on the same nb^2 / eps workload,
    bounded to ~budget_s of CPU time."""
    from oracle import oracle as O  # test infrastructure: baseline leg only

    dh = 1.0 / nb
    dt = eps ** 4 * dh * dh / (8.0 * N.disk_count(eps))
    p = O.params(nb, nb, eps, 1.0, dt, dh, int(test))
    u = O.test_init(p)
    tiles = max(1, nb // 128)  # 128 x 128-node tiles
    t1 = O.run_tiled(p, 1, tiles, tiles, u, nthreads)
    steps = int(max(1, min(20, budget_s / max(t1, 1e-3) - 1)))
    t = O.run_tiled(p, steps, tiles, tiles, u, nthreads)
    rate = nb * nb * steps / t / 1e9
    return {"value": rate, "unit": "Gnode-updates/s", "cores": nthreads, "kind": "port",
            "sample": f"{nb}x{nb} lattice, eps={eps}, test={int(test)}, {steps} step(s) after 1 warm-up step, "
                      f"{tiles}x{tiles} tiles, oracle/nlh_oracle.c run_tiled (-O3 -ffp-contract=off)"}


def workload_name(nb, eps, strong, test, nx, ny) -> str:
    mode = "test mode (manufactured source)" if test else "production step (test=0)"
    if not strong and nb == NB and eps == EPS:
        return f"C2: {nb}x{nb} lattice per GPU, eps={eps}, {mode}"
    if strong:
        return f"{nx}x{ny} lattice in total (strong scaling), eps={eps}, {mode}"
    return f"{nb}x{nb} lattice per GPU, eps={eps}, {mode}"


def read_traffic(kernel_name: str):
    """HBM bytes per stencil launch from the committed rocprofv3 PMC summary
    (FETCH_SIZE doubled per the gfx950 correction + WRITE_SIZE), if that
    summary was taken on the kernel this run launches."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    if d.get("kernel_match") != kernel_name:
        return None
    return d.get("hbm_bytes_per_launch")


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--kernel", default="fast", choices=["fast", "exact"])
    ap.add_argument("--seg-rows", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # secondary workloads (the default line is C2): --eps 32 --lattice 8192 is
    # C4; --lattice 32768 --strong is C3 (total lattice fixed as N grows);
    # --test-mode times the manufactured-solution step and reports its L2
    ap.add_argument("--eps", type=int, default=EPS)
    ap.add_argument("--lattice", type=int, default=NB, help="lattice edge per GPU (weak) or total (--strong)")
    ap.add_argument("--strong", action="store_true")
    ap.add_argument("--test-mode", action="store_true")
    args = ap.parse_args()
    eps, nb = args.eps, args.lattice

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        print(f"--gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    nranks = world

    dist = None
    if nranks > 1:
        import torch.distributed as dist  # control plane only (id broadcast, barrier, max)
        dist.init_process_group("gloo")

    px, py = decomposition(nranks)
    if args.strong:
        if nb % px or nb % py:
            print(f"--lattice {nb} is not divisible by the {px}x{py} block grid", file=sys.stderr)
            return 2
        nx, ny = nb, nb
    else:
        nx, ny = nb * px, nb * py
    dh = 1.0 / nb
    dt = eps ** 4 * dh * dh / (8.0 * N.disk_count(eps))

    comm_id = None
    if nranks > 1:
        obj = [N.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        comm_id = obj[0]

    s = N.Solver(nx, ny, eps, 1.0, dt, dh, test=args.test_mode, kernel=args.kernel, device=local,
                 rank=rank, nranks=nranks, tiles=(px, py), comm_id=comm_id, seg_rows=args.seg_rows)
    s.test_init()
    s.run(args.warmup)
    s.synchronize()

    def barrier():
        s.synchronize()
        if dist is not None:
            dist.barrier()

    barrier()
    # HIP events on the stencil stream bracket the timed region (one pair);
    # the average launch duration below is their span / launches
    s.kernel_timing(True)
    t0 = time.perf_counter()
    s.run(args.steps)
    s.synchronize()
    t1 = time.perf_counter()
    k_ms, k_n = s.kernel_time()
    s.kernel_timing(False)
    barrier()
    elapsed = t1 - t0
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    l2 = s.compute_l2(s.step_index) if args.test_mode else None  # after the timed region
    info = s.info()
    total_nodes = nx * ny
    value = total_nodes * args.steps / elapsed / 1e9
    ms_per_step = elapsed * 1e3 / args.steps
    local_nodes = info.owned_nodes
    # one stencil launch (a "pass") advances steps_per_pass time steps: 2 for
    # the temporally blocked production kernel k_pair, 1 for k_fast / k_exact
    spp = info.steps_per_pass
    kname = info.pass_kernel
    passes = max(k_n // spp, 1)
    avg_launch_s = (k_ms / 1e3) / passes
    # algorithmic bytes per launch = 16 B per node-update x node-updates of one launch
    # + 8 B per node when the fast test mode reads its precomputed L_h[W0]
    bytes_node = BYTES_PER_NODE + (8.0 if args.test_mode and info.kernel == N.KERNEL_FAST else 0.0)
    alg_bytes = bytes_node * local_nodes * spp
    achieved_gbs = alg_bytes / avg_launch_s / 1e9
    fp64_equiv_tflops = 2.0 * info.disk_points * local_nodes * spp / avg_launch_s / 1e12
    # the committed PMC summary was taken on the default C2 workload only
    default_wl = nb == NB and eps == EPS and not args.strong and not args.test_mode
    traffic = read_traffic(kname) if nranks == 1 and default_wl else None

    result = None
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and nranks == 1:
            # bounded sample: at most a 4096^2 lattice of the same eps / mode
            cpu = cpu_baseline(min(16, os.cpu_count() or 1), min(nb, NB), eps, args.test_mode)
        result = {
            "metric": f"Gnode-updates/s (nodes*steps/s) eps={eps} fp64",
            "value": value,
            "unit": "Gnode-updates/s",
            "n_gpus": nranks,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (test_init IC sin(2 pi x) sin(2 pi y); no dataset)",
            "config": {
                "workload": workload_name(nb, eps, args.strong, args.test_mode, nx, ny)
                            + f", {args.kernel} kernel" + (f", {px}x{py} blocks + RCCL ghost exchange" if nranks > 1 else ""),
                "lattice": [nx, ny], "eps": eps, "blocks": [px, py], "test_mode": args.test_mode,
                "disk_points": info.disk_points, "dt": dt, "dh": dh, "kernel": args.kernel,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": kname,
                "steps_per_launch": spp,
                "kernel_avg_us": avg_launch_s * 1e6,
                "kernel_launches_timed": passes,
                "algorithmic_bytes_per_launch": alg_bytes,
                "fp64_direct_sum_equiv_tflops": fp64_equiv_tflops,
                "fp64_direct_sum_equiv_frac": fp64_equiv_tflops / FP64_VEC_PEAK_TFLOPS,
            },
            "cpu_baseline": cpu,
        }
        if l2 is not None:
            result["config"]["l2_error"] = l2  # reference error_l2 at the final step
        print(json.dumps(result), flush=True)
    s.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
