#!/usr/bin/env python3
"""Summarise tools/pmc.sh output for one kernel into the record bench.py reads
as roofline.physical (profiles/pmc/<kernel>__<workload>.json).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 derived metrics).
gfx950 correction (MI355X_MICROARCH.md 'HBM'): FETCH_SIZE reports exactly half
the bytes of wide coalesced streaming reads -> doubled here; WRITE_SIZE is
exact for 16-B-per-lane stores.  SQ_* are per dispatch, summed over the chip.

    python tools/pmc_summary.py DIR KERNEL [--workload KEY --node-updates N --commit SHA --build-id ID]

--build-id: the libnlh build id of the profiled run (bench.py uses a
committed record only when it equals the loaded library's).

KERNEL is the short kernel name (k_pair_split, k_wide, k_fast, k_exact); it
is matched against rocprofv3's demangled names as "KERNEL<".
"""
import argparse
import csv
import glob
import json
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("kernel")
    ap.add_argument("--workload", default=None)
    ap.add_argument("--node-updates", type=float, default=None, help="node-updates per launch")
    ap.add_argument("--commit", default=None)
    ap.add_argument("--build-id", default=None)
    a = ap.parse_args()
    key = a.kernel + "<"
    vals, kdurs = {}, {}
    for f in sorted(glob.glob(os.path.join(a.dir, "p*", "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if key in row["Kernel_Name"]:
                vals.setdefault(row["Counter_Name"], {}).setdefault(row["Kernel_Name"], []).append(
                    float(row["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(a.dir, "p*", "run_kernel_trace.csv"))):
        for row in csv.DictReader(open(f)):
            if key in row["Kernel_Name"]:
                kdurs.setdefault(row["Kernel_Name"], []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    # a "launch" here is one pass: the median of each kernel instance, summed
    # over the instances the pass launches (one for every kernel libnlh has today)
    med = {c: sum(statistics.median(v) for v in per.values()) for c, per in vals.items()}
    durs = [sum(statistics.median(v) for v in kdurs.values())] if kdurs else []
    out = {"kernel_match": a.kernel, "workload": a.workload, "commit": a.commit, "build_id": a.build_id,
           "dispatches_per_counter": {c: sum(len(v) for v in per.values()) for c, per in vals.items()},
           "kernel_instances_per_pass": len(kdurs), "median": med}
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        rd = 2.0 * med["FETCH_SIZE"] * 1024
        wr = med["WRITE_SIZE"] * 1024
        out["hbm_read_bytes_per_launch"] = rd
        out["hbm_write_bytes_per_launch"] = wr
        out["hbm_bytes_per_launch"] = rd + wr
        out["correction"] = "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads), KiB -> bytes"
    if "SQ_INSTS_VALU" in med:
        out["valu_insts_per_launch"] = med["SQ_INSTS_VALU"]
    if a.node_updates:
        out["node_updates_per_launch"] = a.node_updates
        if "hbm_bytes_per_launch" in out:
            out["hbm_bytes_per_node_update"] = out["hbm_bytes_per_launch"] / a.node_updates
        if "valu_insts_per_launch" in out:
            out["valu_lane_ops_per_node_update"] = 64.0 * out["valu_insts_per_launch"] / a.node_updates
    if durs:
        out["profiled_duration_us_median"] = statistics.median(durs) / 1e3
    w = med.get("SQ_WAVE_CYCLES")
    if w:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in med:
                out.setdefault("share_of_wave_cycles", {})[k] = med[k] / w
    if "TCC_HIT_sum" in med:
        out["l2_hit_rate"] = med["TCC_HIT_sum"] / max(1.0, med["TCC_HIT_sum"] + med["TCC_MISS_sum"])
    if "GRBM_GUI_ACTIVE" in med and durs:
        out["effective_clock_ghz"] = med["GRBM_GUI_ACTIVE"] / 8 / (statistics.median(durs))
        if "SQ_LDS_IDX_ACTIVE" in med:
            # LDS-array busy share: cycles summed over the 256 CUs
            out["lds_busy_share"] = med["SQ_LDS_IDX_ACTIVE"] / 256 / (med["GRBM_GUI_ACTIVE"] / 8)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
