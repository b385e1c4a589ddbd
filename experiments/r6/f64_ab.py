#!/usr/bin/env python3
"""Round 6: fp64 LDS ring (4x8:1sl, FCfg::LR + LRC) vs the register ring (4x8:1s) -- in-process
timings, interleaved rounds, random init, L = 512 and 1024 fp64, T = 2 and 3, schedules 1 / 2."""
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    res = {}
    for L, steps in ((512, 60), (1024, 12)):
        sims = {}
        for fuse in (2, 3):
            s = Settings(L=L, precision="Float64", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                         noise=0.1, backend="AMDGPU")
            sims[fuse] = GrayScott(s, init_domain(L, 1, 0), fuse=fuse)
            sims[fuse].init_fields()
        for r in range(2):
            for fuse in (3, 2):
                for cfg in ("4x8:1s", "4x8:1sl"):
                    for sched in (1, 2):
                        sim = sims[fuse]
                        native.fused_select(cfg)
                        native.fused_sched(sched)
                        sim.randomize_fields(seed=2024)
                        sim.set_step(0)
                        sim.iterate(2 * fuse)
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        sim.iterate(steps)
                        torch.cuda.synchronize()
                        dt = time.perf_counter() - t0
                        res.setdefault((L, fuse, cfg, sched), []).append(L ** 3 * steps / dt / 1e6)
            print("L", L, "round", r, "done", flush=True)
        for s in sims.values():
            s.close()
        del sims
        torch.cuda.empty_cache()
    native.fused_unpin()
    for (L, fuse, cfg, sched), v in res.items():
        print(f"L={L} T={fuse} cfg={cfg:8s} sched={sched}  median {statistics.median(v):9.0f}  "
              f"[{min(v):.0f}, {max(v):.0f}] MLUPS", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
