#!/usr/bin/env python3
"""In-process A/B tuning of fused-kernel configurations (interleaved rounds on ONE device, as
the CDNA methodology rules require; separate processes/boxes differ by +-10 %).

  python scripts/tune_inproc.py --L 256 512 --fuse 2 3 --cfg "" 8x4:3 4x12:2 --rounds 3
"""
import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, nargs="+", default=[256, 512])
    ap.add_argument("--fuse", type=int, nargs="+", default=[2, 3])
    ap.add_argument("--cfg", nargs="+", default=[""])
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--precision", default="Float32")
    ap.add_argument("--out", default="")
    ap.add_argument("--noise", type=float, default=0.1)
    ap.add_argument("--sched", type=int, nargs="+", default=[0])
    ap.add_argument("--init", choices=["seed", "random"], default="seed",
                    help="random: every timed run starts from the same u, v ~ U[0,1) state "
                         "(the benchmark's; power-limited regime), after --warmup steps")
    ap.add_argument("--warmup", type=int, default=12)
    a = ap.parse_args()
    import torch
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    results = {}
    for L in a.L:
        sims = {}
        for fuse in a.fuse:
            s = Settings(L=L, precision=a.precision, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                         noise=a.noise, backend="AMDGPU")
            sim = GrayScott(s, init_domain(L, 1, 0), fuse=fuse)
            sim.init_fields()
            sims[fuse] = sim
        for r in range(a.rounds):
            for fuse, sim in sims.items():
                for cfg in a.cfg:
                    for sched in a.sched:
                        native.fused_select(cfg)
                        native.fused_sched(sched)
                        if a.init == "random":
                            sim.randomize_fields(seed=2024)
                            sim.set_step(0)
                        sim.iterate(a.warmup)
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        sim.iterate(a.steps)
                        torch.cuda.synchronize()
                        dt = time.perf_counter() - t0
                        key = (f"L={L} fuse={fuse} cfg={cfg or 'default'} sched={sched}"
                               f"{' random' if a.init == 'random' else ''}")
                        results.setdefault(key, []).append(L ** 3 * a.steps / dt / 1e6)
        for sim in sims.values():
            sim.close()
        del sims
        torch.cuda.empty_cache()
    native.fused_select("")
    native.fused_sched(0)
    rows = []
    for k, v in results.items():
        rows.append({"config": k, "median_mlups": statistics.median(v), "min": min(v), "max": max(v)})
        print(f"{k:40s} median {statistics.median(v):10.0f}  [{min(v):.0f}, {max(v):.0f}] MLUPS",
              flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
