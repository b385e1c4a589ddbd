#!/usr/bin/env python3
"""Round 6 soak of the hand-counted LDS-DMA waits: long runs through the LDS-ring shapes (T=4
4x12:1sfl / 1sl, T=2 4x12:2sfl, fp64 4x8:1sl) against the register-ring shapes (no LDS-DMA), bit for
bit, over hundreds of steps, repeated.  Step counts are multiples of every depth used (every
fused depth is bit-identical; a single-step remainder would run the separate k_step1 kernel,
whose evaluation order differs in the last bits)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(L, steps, fuse, cfg, prec="Float32", sched=None):
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    native.fused_unpin()
    if cfg is not None:
        native.fused_select(cfg)
        native.fused_sched(2 if sched is None else sched)
    s = Settings(L=L, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend="AMDGPU", seed=11)
    sim = GrayScott(s, init_domain(L, 1, 0), fuse=fuse)
    try:
        sim.init_fields()
        sim.randomize_fields(seed=5)
        sim.iterate(steps)
        out = sim.get_fields()
        ch = sim.fused_choice()
    finally:
        sim.close()
        native.fused_unpin()
    return out, ch


def main():
    import numpy as np
    bad = 0
    cases = [  # (L, steps, prec, [(label, fuse, cfg, sched)])
        (200, 600, "Float32", [("T=4 tuned (LR)", 4, None, None), ("T=2 4x12:2sfl", 2, "4x12:2sfl", 0),
                               ("T=4 4x12:1sl s1", 4, "4x12:1sl", 1)]),
        (256, 600, "Float32", [("T=4 tuned (LR)", 4, None, None), ("T=2 4x12:2sfl", 2, "4x12:2sfl", 2),
                               ("T=3 4x12:1sfl", 3, "4x12:1sfl", 1)]),
        (512, 240, "Float32", [("T=4 tuned (LR)", 4, None, None), ("T=3 4x12:2sl", 3, "4x12:2sl", 2)]),
        (200, 300, "Float64", [("T=3 4x8:1sl", 3, "4x8:1sl", 0), ("T=2 4x8:1sl", 2, "4x8:1sl", 2)]),
        (320, 300, "Float64", [("T=3 4x8:1sl", 3, "4x8:1sl", 1)]),
    ]
    for rep in range(2):
        for L, steps, prec, variants in cases:
            ref, _ = run(L, steps, 3, "4x12:1s" if prec == "Float32" else "4x8:1s", prec)
            for label, fuse, cfg, sched in variants:
                a, ch = run(L, steps, fuse, cfg, prec, sched)
                eq = np.array_equal(a[0], ref[0]) and np.array_equal(a[1], ref[1])
                bad += 0 if eq else 1
                nd = int(((a[0] != ref[0]) | (a[1] != ref[1])).sum())
                print(f"rep {rep} L={L} {prec} {steps} steps {label:18s} "
                      f"({ {k: v[0] for k, v in ch.items()} }): "
                      f"{'bitwise' if eq else f'DIFF in {nd} cells'}", flush=True)
    print("soak failures:", bad)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
