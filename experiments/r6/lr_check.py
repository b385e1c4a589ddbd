#!/usr/bin/env python3
"""Round 6: the LDS-ring (FCfg::LR) shapes and the T = 4 entry -- bitwise against the register-
ring production shape, then in-process timings (interleaved rounds, random init, L = 512).

  python experiments/r6/lr_check.py [--check-only] [--steps 120]
"""
import argparse
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def make(L, fuse, noise=0.1):
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    s = Settings(L=L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                 noise=noise, backend="AMDGPU")
    sim = GrayScott(s, init_domain(L, 1, 0), fuse=fuse)
    sim.init_fields()
    return sim


def run(sim, cfg, sched, steps, seed=2024):
    from grayscott_amd.ops import native
    native.fused_select(cfg)
    native.fused_sched(sched)
    sim.randomize_fields(seed=seed)
    sim.set_step(0)
    sim.iterate(steps)
    sim.synchronize()
    return sim.get_fields()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--check-only", action="store_true")
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--L", type=int, nargs="+", default=[512])
    ap.add_argument("--cases", nargs="+", default=[
        "3:4x12:1s", "3:4x12:2s", "3:4x12:1sl", "3:4x12:2sl", "2:4x12:1s", "2:4x12:2sl",
        "2:4x12:3sl", "4:4x12:1sl"])
    a = ap.parse_args()
    import numpy as np
    import torch
    from grayscott_amd.ops import native
    bad = 0
    for L in (200, 256):
        sims = {n: make(L, n) for n in (2, 3, 4)}
        ref = run(sims[3], "4x12:2s", 2, 12)
        for fuse, cfg, sched in [(3, "4x12:1sl", 0), (3, "4x12:1sl", 2), (3, "4x12:2sl", 1),
                                 (3, "4x12:1sfl", 2), (3, "4x12:2sfl", 2), (2, "4x12:2sl", 2),
                                 (2, "4x12:3sl", 0), (2, "4x12:1sfl", 2), (4, "4x12:1sl", 0),
                                 (4, "4x12:1sl", 1), (4, "4x12:1sl", 2), (4, "4x12:1sfl", 2),
                                 (2, "4x12:1s", 2), (4, "", 2)]:
            got = run(sims[fuse], cfg, sched, 12)
            du = float(np.max(np.abs(got[0] - ref[0])))
            dv = float(np.max(np.abs(got[1] - ref[1])))
            eq = bool(np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]))
            bad += 0 if eq else 1
            print(f"check L={L} T={fuse} cfg={cfg or 'default'} sched={sched}: "
                  f"{'bitwise' if eq else 'DIFF'} max|du|={du:.3g} max|dv|={dv:.3g}", flush=True)
        for s in sims.values():
            s.close()
        del sims
        torch.cuda.empty_cache()
    print("check failures:", bad, flush=True)
    if a.check_only or bad:
        return 1 if bad else 0
    res = {}
    for L in a.L:
        sims = {n: make(L, n) for n in (2, 3, 4)}
        cases = [(int(c.split(":", 1)[0]), c.split(":", 1)[1]) for c in a.cases]
        for r in range(a.rounds):
            for fuse, cfg in cases:
                for sched in (1, 2):
                    sim = sims[fuse]
                    native.fused_select(cfg)
                    native.fused_sched(sched)
                    sim.randomize_fields(seed=2024)
                    sim.set_step(0)
                    sim.iterate(12)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    sim.iterate(a.steps)
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                    res.setdefault((L, fuse, cfg, sched), []).append(L ** 3 * a.steps / dt / 1e6)
            print("round", r, "done", flush=True)
        for s in sims.values():
            s.close()
        del sims
        torch.cuda.empty_cache()
    native.fused_select("")
    native.fused_sched(0)
    for (L, fuse, cfg, sched), v in res.items():
        print(f"L={L} T={fuse} cfg={cfg:10s} sched={sched}  median {statistics.median(v):9.0f}  "
              f"[{min(v):.0f}, {max(v):.0f}] MLUPS  ({a.steps} steps, random init)", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
