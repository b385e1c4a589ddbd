#!/usr/bin/env python3
"""Bitwise digest of a few fused steps per kernel configuration (ablation A/Bs whose variants
must be exact: same digest as the production configuration).  GS_HIP_VARIANT=abl for the
ablation build.

  GS_HIP_VARIANT=abl python scripts/abl_digest.py --cfg 4x12:1s 4x12:1s-abl4
"""
import argparse
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cfg", nargs="+", required=True)
    ap.add_argument("--L", type=int, default=256)
    ap.add_argument("--steps", type=int, default=9)
    ap.add_argument("--sched", type=int, default=2)
    a = ap.parse_args()
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    for cfg in a.cfg:
        native.fused_select(cfg)
        native.fused_sched(a.sched)
        s = Settings(L=a.L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                     noise=0.1, backend="AMDGPU")
        sim = GrayScott(s, init_domain(a.L, 1, 0), fuse=3)
        sim.init_fields()
        sim.randomize_fields(seed=5)
        sim.iterate(a.steps)
        u, v = sim.get_fields()
        print(f"{cfg:16s} {hashlib.sha1(u.tobytes() + v.tobytes()).hexdigest()}", flush=True)
        sim.close()


if __name__ == "__main__":
    main()
