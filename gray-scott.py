#!/usr/bin/env python3
"""CLI entry script (reference gray-scott.jl): runs the simulation and reports wall time.

    python gray-scott.py settings-files.toml
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 gray-scott.py settings-files.toml
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from grayscott_amd.driver import julia_main  # noqa: E402

if __name__ == "__main__":
    t0 = time.perf_counter()
    rc = julia_main(sys.argv[1:])
    if int(os.environ.get("RANK", "0")) == 0:
        print(f"{time.perf_counter() - t0:.6f} seconds", file=sys.stderr)
    sys.exit(rc)
