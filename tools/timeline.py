#!/usr/bin/env python3
"""Per-pass kernel timeline from a rocprofv3 --kernel-trace CSV: for each
launch its queue, start/end relative to the first traced stencil launch, and
a summary of gaps and overlap between the interior and the band launches.
    python tools/timeline.py run_kernel_trace.csv [--last 12]
"""
import csv
import sys


def short(name):
    n = name.split("(")[0].replace("void ", "").replace("nlh::", "")
    return n[:40]


def main():
    path = sys.argv[1]
    last = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--last" else 16
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]),
                         short(r["Kernel_Name"]), int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    rows = rows[-last:]
    t0 = rows[0][0]
    for s, e, q, n, g in rows:
        print(f"q{q:<3d} {(s - t0) / 1e3:9.2f} {(e - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f} us  wg={g:<6d} {n}")


if __name__ == "__main__":
    main()
