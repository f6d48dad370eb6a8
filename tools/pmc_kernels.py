"""Summarise rocprofv3 --pmc passes per kernel symbol (tools only).

Usage: python3 tools/pmc_kernels.py DIR   (DIR/p*/.../run_counter_collection.csv)
Prints one JSON object: kernel -> {counter: mean per dispatch, "dispatches": n}.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def main(d: str) -> None:
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            per = defaultdict(float)
            names = {}
            for r in csv.DictReader(fh):
                key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Counter_Name"])
                per[key] += float(r["Counter_Value"])
                names[key[0]] = r["Kernel_Name"]
            for (disp, cname), v in per.items():
                kn = names[disp]
                m = re.search(r"k_pair_split<(\d+), (\d+), (\d+), (\d+), (\w+), (\d+)>", kn)
                short = f"E{m.group(1)}_abl{m.group(3)}_opt{m.group(6)}" if m else kn[:60]
                acc[short][cname].append(v)
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
