#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs (scripts/profile_kernels.sh output) per kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict


def _key(name: str) -> str:
    """Kernel name without its parameter list (the template arguments are kept: they tell the
    fused kernel's configurations apart)."""
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    depth = 0
    for i, ch in enumerate(name):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return name[:i]
    return name


def main(root):
    acc = defaultdict(lambda: defaultdict(float))
    vals = defaultdict(lambda: defaultdict(list))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = _key(row["Kernel_Name"])
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                cnt[k][row["Counter_Name"]] += 1
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(root, "stats", "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                durs[_key(row["Name"])] = [int(row["Calls"]), float(row["AverageNs"])]
    for k, d in acc.items():
        print(f"== {k}  calls/avg_ns={durs.get(k)}")
        for c in sorted(d):
            n = max(1, cnt[k][c])
            v = sorted(vals[k][c])
            med = v[len(v) // 2] if v else 0.0
            print(f"   {c:28s} per-dispatch mean {d[c] / n:.4g}  median {med:.4g}  (n={n})")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
