#!/usr/bin/env python3
"""Round 6 diagnosis: fp64 LDS ring (4x8:1sl) vs register ring (4x8:1s), per (L, T, sched):
mismatch count and where the mismatching cells lie (z / y / x ranges, first steps)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def run(L, fuse, sched, cfg, steps):
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    native.fused_select(cfg)
    native.fused_sched(sched)
    s = Settings(L=L, precision="Float64", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                 noise=float(os.environ.get("NOISE", "0.1")), backend="AMDGPU", seed=31)
    sim = GrayScott(s, init_domain(L, 1, 0), fuse=fuse)
    try:
        sim.init_fields()
        sim.randomize_fields(seed=3)
        sim.iterate(steps)
        return sim.get_fields()
    finally:
        sim.close()


def main():
    import numpy as np
    cases = [(200, 3, 2, 13), (256, 3, 1, 13), (200, 2, 0, 9), (96, 3, 2, 13), (256, 2, 2, 9)]
    cases = cases * int(os.environ.get("REPEAT", "3"))
    if os.environ.get("FIRST"):
        cases = [(200, 2, 0, 2), (200, 2, 2, 2), (200, 2, 0, 9), (256, 2, 2, 2), (200, 3, 0, 3),
                 (200, 3, 2, 3), (96, 3, 2, 3), (64, 2, 2, 2)]
    if os.environ.get("GOLD"):
        # the failing sequence, each shape against the CPU golden model (fp64, 1e-12)
        from grayscott_amd.models.grayscott import GrayScott
        from grayscott_amd.parallel.decomp import init_domain
        from grayscott_amd.utils.config import Settings
        s = Settings(L=200, precision="Float64", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                     noise=0.1, backend="CPU", seed=31)
        c = GrayScott(s, init_domain(200, 1, 0), fuse=1)
        c.init_fields()
        c.randomize_fields(seed=3)
        c.iterate(9)
        gold = c.get_fields()
        c.close()
        cfgs = os.environ.get("CFGS", "4x8:1s,4x8:1sl,4x8:1s,4x8:1sl").split(",")
        for rep in range(int(os.environ.get("REPS", "3"))):
            for L, fuse, sched, steps in [(200, 3, 2, 13), (256, 3, 1, 13)]:
                run(L, fuse, sched, "4x8:1s", steps)
                run(L, fuse, sched, "4x8:1sl", steps)
            for cfg in cfgs:
                a = run(200, 2, 0, cfg, 9)
                err = max(float(np.abs(a[0] - gold[0]).max()), float(np.abs(a[1] - gold[1]).max()))
                bad = (np.abs(a[0] - gold[0]) > 1e-12) | (np.abs(a[1] - gold[1]) > 1e-12)
                print(f"gold rep {rep} {cfg}: max err {err:.3g}, {int(bad.sum())} cells > 1e-12",
                      flush=True)
        cases = []
    if os.environ.get("SELF"):
        # which shape is nondeterministic: each run twice against itself
        for L, fuse, sched, steps in [(200, 2, 0, 9)] * 4:
            for cfg in ("4x8:1s", "4x8:1sl"):
                a = run(L, fuse, sched, cfg, steps)
                b = run(L, fuse, sched, cfg, steps)
                bad = (a[0] != b[0]) | (a[1] != b[1])
                print(f"self {cfg} L={L} T={fuse} sched={sched}: {int(bad.sum())} mismatches",
                      flush=True)
        cases = []
    for L, fuse, sched, steps in cases:
        a = run(L, fuse, sched, "4x8:1s", steps)
        b = run(L, fuse, sched, "4x8:1sl", steps)
        bad = (a[0] != b[0]) | (a[1] != b[1])
        n = int(bad.sum())
        msg = f"L={L} T={fuse} sched={sched} steps={steps}: {n} mismatches"
        if n:
            z, y, x = np.nonzero(bad)
            zs = np.unique(z)
            msg += (f"; z {zs[:12].tolist()}{'...' if len(zs) > 12 else ''} ({len(zs)} planes)"
                    f" y [{y.min()},{y.max()}] x [{x.min()},{x.max()}]"
                    f" nan_lr={int(np.isnan(b[0]).sum())}")
        print(msg, flush=True)
    from grayscott_amd.ops import native
    native.fused_unpin()


if __name__ == "__main__":
    main()
