#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV by kernel family.

    tools/trace_summary.py KERNEL_TRACE_CSV [--passes P] [--ranks V]

Prints one JSON object: per family (k_pair_split, k_wide, k_prefix_rt,
k_copies, RCCL kernels, ...) the launch count, total and mean duration, and
-- with --passes (stencil passes in the traced run) and --ranks (virtual
ranks the process ran, NLH_VIRTUAL_RANKS) -- the per-pass and per-rank-per-pass
figures the multi-GPU prediction in DESIGN.md uses.  Kernel durations come
from the trace's Start/End timestamps (ns)."""
import argparse
import csv
import json
import re
from collections import defaultdict


def family(name: str) -> str:
    n = name.split("(")[0]
    m = re.search(r"nlh::(k_\w+?)(?:<|$)", n) or re.search(r"\b(k_\w+?)(?:<|$)", n)
    if m:
        return m.group(1)
    low = n.lower()
    if "nccl" in low or "rccl" in low:
        return "rccl"
    return n[:60]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--passes", type=int, default=0)
    ap.add_argument("--ranks", type=int, default=1)
    args = ap.parse_args()
    fam = defaultdict(list)
    t0, t1 = None, None
    for row in csv.DictReader(open(args.trace)):
        s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
        fam[family(row["Kernel_Name"])].append((s, e, int(row.get("Grid_Size", 0) or 0)))
        t0 = s if t0 is None else min(t0, s)
        t1 = e if t1 is None else max(t1, e)
    out = {"trace": args.trace, "span_ms": (t1 - t0) / 1e6 if t0 is not None else 0.0, "families": {}}
    for f, v in sorted(fam.items(), key=lambda kv: -sum(e - s for s, e, _ in kv[1])):
        tot = sum(e - s for s, e, _ in v) / 1e3
        d = {"launches": len(v), "total_us": tot, "mean_us": tot / len(v)}
        if args.passes:
            d["us_per_pass"] = tot / args.passes
            d["us_per_rank_per_pass"] = tot / args.passes / max(1, args.ranks)
        out["families"][f] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
