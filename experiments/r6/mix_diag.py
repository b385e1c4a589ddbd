#!/usr/bin/env python3
"""Round 6 diagnosis: L=200 fp64, an odd step count -- the planner's [3.., 2, 2] passes vs T=3 greedy
passes + one single step vs the CPU golden model (fp64: 1e-12), and variants isolating the pass mix."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import numpy as np
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    L, steps = int(os.environ.get("L", "200")), int(os.environ.get("STEPS", "301"))
    prec = os.environ.get("PREC", "Float64")

    def make(backend, fuse=None):
        s = Settings(L=L, precision=prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                     backend=backend, seed=11)
        sim = GrayScott(s, init_domain(L, 1, 0), fuse=fuse)
        sim.init_fields()
        sim.randomize_fields(seed=5)
        return sim

    c = make("CPU", 1)
    c.iterate(steps)
    gold = c.get_fields()
    c.close()

    def check(name, sim, chunks):
        for n in chunks:
            sim.iterate(n)
        u, v = sim.get_fields()
        sim.close()
        d = max(float(np.abs(u - gold[0]).max()), float(np.abs(v - gold[1]).max()))
        nd = int(((np.abs(u - gold[0]) > 1e-10) | (np.abs(v - gold[1]) > 1e-10)).sum())
        print(f"{name:46s} max|d| vs CPU {d:.3e}  cells > 1e-10: {nd}", flush=True)

    tol_steps = steps
    sim = make("AMDGPU")
    print("default plan:", sim.engine.plan_passes(steps), "choice", sim.fused_choice(), flush=True)
    check("default (planner)", sim, [steps])
    sim = make("AMDGPU", 3)
    check("fuse=3 greedy (T=3 passes + remainder)", sim, [steps])
    sim = make("AMDGPU", 2)
    check("fuse=2 greedy (T=2 passes + remainder)", sim, [steps])
    sim = make("AMDGPU")
    sim.engine.set_plan(False)
    check("default H, planner off (greedy at depth)", sim, [steps])
    sim = make("AMDGPU", 3)
    check("fuse=3, chunks of 2 steps", sim, [2] * (steps // 2) + [steps % 2])
    sim = make("AMDGPU", 3)
    check("fuse=3, chunks of 1 step", sim, [1] * steps)
    native.fused_unpin()


if __name__ == "__main__":
    main()
