#!/usr/bin/env python3
"""Round 6: is L=64 host-bound?  Time sim.iterate(n)'s return (host enqueue) against the time to
the device's completion, for the autotuned set-up at L=64 / 96 / 128."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    for L in (64, 96, 128):
        s = Settings(L=L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                     noise=0.1, backend="AMDGPU")
        sim = GrayScott(s, init_domain(L, 1, 0))
        sim.init_fields()
        sim.randomize_fields(seed=1)
        sim.iterate(60)
        sim.synchronize()
        torch.cuda.synchronize()
        for n in (600, 3000):
            t0 = time.perf_counter()
            sim.iterate(n)
            t1 = time.perf_counter()
            sim.synchronize()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            plan = sim.engine.plan_passes(n)
            print(f"L={L} n={n} passes={len(plan) or '?'} enqueue {1e6 * (t1 - t0) / n:.2f} us/step, "
                  f"total {1e6 * (t2 - t0) / n:.2f} us/step -> {L ** 3 / ((t2 - t0) / n) / 1e6:.0f} MLUPS",
                  flush=True)
        sim.close()


if __name__ == "__main__":
    main()
