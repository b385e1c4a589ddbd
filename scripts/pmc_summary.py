#!/usr/bin/env python3
"""Summarise rocprofv3 counter CSVs (scripts/profile_kernels.sh output) per kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    acc = defaultdict(lambda: defaultdict(float))
    cnt = defaultdict(lambda: defaultdict(int))
    for f in glob.glob(os.path.join(root, "g*", "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].split("(")[0][:70]
                acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
                cnt[k][row["Counter_Name"]] += 1
    durs = defaultdict(list)
    for f in glob.glob(os.path.join(root, "stats", "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                durs[row["Name"].split("(")[0][:70]] = [int(row["Calls"]), float(row["AverageNs"])]
    for k, d in acc.items():
        print(f"== {k}  calls/avg_ns={durs.get(k)}")
        for c in sorted(d):
            n = max(1, cnt[k][c])
            print(f"   {c:28s} per-dispatch {d[c] / n * (1 if 'SQ_' not in c else 1):.4g}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
