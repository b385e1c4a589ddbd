#!/usr/bin/env python3
"""Per-pass timing of the fused kernel against the field's data (profiles/r2_power_probe.txt).

The same T-step pass is timed (hipEvents around each pass) on different states of one L^3 grid:
  seed    the reference init (u = 1, v = 0 except the 13^3 cube): nearly constant data
  random  u, v ~ U[0, 1) (BASELINE.json's benchmark init)
  zero    u = v = 0 plus noise (only the noise term varies)
and, for random, the passes that follow, to see how the speed evolves with the state.

  python scripts/power_probe.py [--L 512] [--passes 60]
  python scripts/power_probe.py --matrix     # seed vs random for several kernel variants
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--passes", type=int, default=60)
    ap.add_argument("--noise", type=float, default=0.1)
    ap.add_argument("--matrix", action="store_true")
    a = ap.parse_args()
    import torch

    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    def make(noise, fuse=None):
        s = Settings(L=a.L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                     noise=noise, backend="AMDGPU")
        sim = GrayScott(s, init_domain(a.L, 1, 0), fuse=fuse)
        sim.init_fields()
        return sim

    def timed(sim, n, k):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * n)]
        for i in range(n):
            ev[2 * i].record()
            sim.iterate(k)
            ev[2 * i + 1].record()
        torch.cuda.synchronize()
        return [ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(n)]

    if a.matrix:
        # (label, noise, fuse, fused-kernel config or None = autotuned)
        variants = [("T3", a.noise, 3, None), ("T3-nonoise", 0.0, 3, None),
                    ("T2", a.noise, 2, None),
                    # ablations: GS_HIP_VARIANT=abl (make ablation) only; results are wrong
                    ("T3-L2loads(wrong)", a.noise, 3, "4x12:2s-abl2"),
                    ("T3-nobarrier(wrong)", a.noise, 3, "4x12:2s-abl1"),
                    ("T3-4x12:1s", a.noise, 3, "4x12:1s")]
        for label, noise, fuse, cfg in variants:
            sim = make(noise, fuse)
            if cfg is not None:
                try:
                    native.fused_select(cfg)
                    native.fused_sched(2)
                except ValueError:
                    print(f"{label:22s} not in this build", flush=True)
                    sim.close()
                    continue
            seed = timed(sim, 8, fuse)
            sim.randomize_fields(seed=2024)
            sim.set_step(0)
            rnd = timed(sim, 8, fuse)
            ms, mr = statistics.median(seed[2:]), statistics.median(rnd)
            cells = a.L ** 3 * fuse
            print(f"{label:22s} seed {ms:7.1f} us/pass ({cells / ms / 1e0:9.0f} MLUPS)  random "
                  f"{mr:7.1f} us/pass ({cells / mr:9.0f} MLUPS)  ratio {mr / ms:5.3f}", flush=True)
            if cfg is not None:
                native.fused_select("")
            sim.close()
            torch.cuda.synchronize()
        return

    sim = make(a.noise)
    k = sim.fuse

    def run(tag, n):
        ts = timed(sim, n, k)
        st = sim.global_stats()
        print(f"{tag:8s} T={k} us/pass: " + " ".join(f"{t:.0f}" for t in ts), flush=True)
        print(f"{tag:8s} mean_u={st['mean_u']:.4f} mean_v={st['mean_v']:.4f} "
              f"min_v={st['min_v']:.3g} max_v={st['max_v']:.3g}", flush=True)

    run("seed", 10)
    sim.randomize_fields(seed=2024)
    sim.set_step(0)
    run("random", a.passes)
    run("random+", a.passes)
    sim.randomize_fields(seed=2024, lo=0.0, hi=1e-30)
    run("zero", 10)
    sim.close()


if __name__ == "__main__":
    main()
