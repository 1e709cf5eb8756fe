"""Per-shape summary of a rocprofv3 --kernel-trace run (scripts/gpu_round.sh, bench.py --profile-only).

Usage: python scripts/trace_summary.py <dir with run_kernel_trace.csv> <out.csv>

rocprofv3's --stats summary averages every launch of one kernel symbol, whatever its grid.  This
groups the sd:: launches by (kernel, grid size) and, for each group, by the kernel that ran just
before it on the same queue: a draw launched right after another draw is the bench's back-to-back
roofline loop; one after the verify's kernels is a step's draw.  Durations are End - Start (ns).
"""
from __future__ import annotations

import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    return name.split("(")[0].replace("void ", "")


def grid(row) -> str:
    if "Grid_Size" in row and row["Grid_Size"]:
        return row["Grid_Size"]
    return "x".join(row.get(f"Grid_Size_{a}", "1") or "1" for a in "XYZ")


def main():
    src, out = sys.argv[1], sys.argv[2]
    paths = glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True)
    rows = []
    for p in paths:
        with open(p) as f:
            rows += list(csv.DictReader(f))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    prev_on_queue = {}
    groups = defaultdict(list)
    for r in rows:
        name = short(r["Kernel_Name"])
        q = r.get("Queue_Id", "0")
        prev = prev_on_queue.get(q)
        prev_on_queue[q] = name
        if "sd::" not in name:
            continue
        fam = "after_same" if prev == name else "after_other"
        groups[(name, grid(r), fam)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "grid", "predecessor", "launches", "mean_ns", "median_ns", "min_ns", "max_ns"])
        for (name, g, fam), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, g, fam, len(d), f"{statistics.mean(d):.0f}", f"{statistics.median(d):.0f}",
                        min(d), max(d)])
    print(open(out).read())


if __name__ == "__main__":
    main()
