#!/usr/bin/env python3
"""Summarise tools/pmc.sh output for one kernel (default: the fast stencil).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (rocprofv3 derived metrics).
gfx950 correction (MI355X_MICROARCH.md 'HBM'): FETCH_SIZE reports exactly half
the bytes of wide coalesced streaming reads -> doubled here; WRITE_SIZE is
exact for 16-B-per-lane stores.  Usage:
    python tools/pmc_summary.py gpurun_out/pmc1 [kernel-substring] > summary.json
"""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    d = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "k_fast"
    vals = {}
    durs = []
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if key not in row["Kernel_Name"]:
                continue
            vals.setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_kernel_trace.csv"))):
        for row in csv.DictReader(open(f)):
            if key in row["Kernel_Name"]:
                durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    med = {k: statistics.median(v) for k, v in vals.items()}
    out = {"kernel_match": key, "dispatches_per_counter": {k: len(v) for k, v in vals.items()},
           "median": med}
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        rd = 2.0 * med["FETCH_SIZE"] * 1024
        wr = med["WRITE_SIZE"] * 1024
        out["hbm_read_bytes_per_launch"] = rd
        out["hbm_write_bytes_per_launch"] = wr
        out["hbm_bytes_per_launch"] = rd + wr
        out["correction"] = "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads), KiB -> bytes"
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
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
