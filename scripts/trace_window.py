#!/usr/bin/env python3
"""Kernel timeline of a bench.py run under rocprofv3 --kernel-trace: the dispatches between the
last autotuning launch and the first k_stats (the timed window plus the warm-up), with start
offsets, durations and the gaps between them, then the per-kernel totals of that window."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("void ", "")
    if "k_fused<" in n:
        import re
        m = re.search(r"FCfg<(\w+), (\d+), (\d+), (\d+), (\d+),.*?(\d+)>, \w+>", n)
        return f"k_fused T={m.group(2)} {m.group(3)}x{m.group(4)}:{m.group(5)} opt{m.group(6)}" if m else n[:40]
    return n.split("(")[0].split("<")[0][:40]


def main(root):
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    stats = [i for i, r in enumerate(rows) if "k_stats" in r[2]]
    end = stats[0] if stats else len(rows)
    # the window: the 40 dispatches before the first k_stats (warm-up + timed region)
    beg = max(0, end - 40)
    t0 = rows[beg][0]
    prev = None
    tot = defaultdict(float)
    for s, e, n in rows[beg:end]:
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        print(f"{(s - t0) / 1e3:10.1f} us  {(e - s) / 1e3:8.1f} us  gap {gap:6.1f}  {short(n)}")
        tot[short(n)] += (e - s) / 1e3
        prev = e
    print("# totals over the window:")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"#   {v:9.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
