#!/usr/bin/env python3
"""Register / LDS / scratch usage of every fused-kernel instantiation in the built library.

Reads the gfx950 code object's AMDHSA metadata (llvm-readelf --notes) -- no GPU needed.  Used
to check that a kernel change keeps the hot configurations within their occupancy budget
(fp32 4x12 T=3: <= 128 VGPRs, i.e. a 12-wave workgroup plus a 4-wave one per CU) and spill-free.

  python scripts/kernel_resources.py [grayscott_amd/_lib/libgs_hip.so] [--all]
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fatbin import LLVM, code_objects  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def notes(lib: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        return "".join(subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                                      capture_output=True, text=True).stdout
                       for co in code_objects(lib, d))


def kernels(text: str, everything: bool = False):
    rows = []
    for b in text.split("- .agpr_count")[1:]:
        name = re.search(r"\.name:\s+(\S+)", b).group(1)
        if not everything and "k_fused" not in name:
            continue

        def f(key):
            m = re.search(rf"\.{key}:\s+(\d+)", b)
            return int(m.group(1)) if m else -1
        rows.append((name, f("vgpr_count"), f("sgpr_count"), f("group_segment_fixed_size"),
                     f("private_segment_fixed_size"), f("vgpr_spill_count"),
                     f("sgpr_spill_count")))
    dem = subprocess.run(["c++filt"], input="\n".join(r[0] for r in rows), capture_output=True,
                         text=True).stdout.split("\n")
    out = []
    for r, d in zip(rows, dem):
        m = re.search(r"FCfg<(.*?)>", d)
        tag = "G " if "k_fused_gated" in d else ""  # the gated pass's entry (gate.hpp)
        out.append((((tag + m.group(1)) if m else d)[:80],) + r[1:])
    return out


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(ROOT, "grayscott_amd", "_lib", "libgs_hip.so")
    print(f"{'configuration':<58} {'vgpr':>5} {'sgpr':>5} {'lds':>7} {'scratch':>7} "
          f"{'vspill':>6} {'sspill':>6}")
    for r in kernels(notes(lib), "--all" in sys.argv):
        print(f"{r[0]:<58} {r[1]:>5} {r[2]:>5} {r[3]:>7} {r[4]:>7} {r[5]:>6} {r[6]:>6}")


if __name__ == "__main__":
    main()
