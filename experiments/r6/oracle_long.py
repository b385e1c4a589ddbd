#!/usr/bin/env python3
"""Round 6: the production path at production size over longer horizons
against the independent PyTorch fp32 oracle (ops/reference.py run_torch): L=512 fp32, random
init, the default single-rank set-up (planner: T=4 / T=3 passes), 60 / 200 / 400 steps; max and
mean |d| and the global statistics."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import reference as ref
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings
    phys = dict(F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1)
    for L, steps in ((512, 60), (512, 200), (512, 400), (256, 1000)):
        s = Settings(L=L, precision="Float32", noise=0.1, backend="AMDGPU", seed=2024, **phys)
        sim = GrayScott(s, init_domain(L, 1, 0))
        try:
            sim.init_fields()
            plan = sim.engine.plan_passes(steps)
            sim.randomize_fields(seed=7)
            sim.iterate(steps)
            u, v = sim.get_fields_device()
            torch.cuda.synchronize()
        finally:
            sim.close()
        ou, ov = ref.run_torch(L, steps, noise_amp=0.1, seed=2024, dtype=torch.float32,
                               device="cuda", init_seed=7, **phys)
        d = [(u - ou).abs(), (v - ov).abs()]
        dmax = max(float(x.max()) for x in d)
        dmean = max(float(x.double().mean()) for x in d)
        st = [float(a.double().mean()) for a in (u, ou, v, ov)]
        print(f"L={L} steps={steps} plan={sorted(set(plan))} x{len(plan)}: max|d| {dmax:.3e} "
              f"mean|d| {dmean:.3e}  mean u {st[0]:.7f} / {st[1]:.7f}  mean v {st[2]:.7f} / "
              f"{st[3]:.7f}", flush=True)
        del u, v, ou, ov, d
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
