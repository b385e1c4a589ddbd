#!/usr/bin/env python3
"""Kernel-side cost of the comm/compute-overlap split on ONE MI355X (no communication).

For a z-slab sub-domain (what one rank of an N-GPU 1x1xN run owns) it times, per k-step pass:
  full   -- one fused launch over all nz planes (the non-overlapped pass),
  inner  -- the launch over planes [k, nz-k) (runs while the halos are in flight),
  shell  -- the launch over the two k-plane boundary slabs (runs after they land).
The overlapped pass costs shell + max(inner, exchange); the plain one full + exchange.
With --packed the sub-domain is one rank of the balanced grid (neighbours on every side):
inner = the inner x-y tiles x planes [k, nz-k), shell = the z end slabs + the ring tiles.

  python scripts/bench_overlap_split.py --nz 64 128 256 --k 2 3
  python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 2 3
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--nz", type=int, nargs="+", default=[64, 128, 256])
    ap.add_argument("--k", type=int, nargs="+", default=[2, 3])
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--out", default="")
    ap.add_argument("--packed", action="store_true")
    ap.add_argument("--one-sided", action="store_true",
                    help="packed: the rank of a non-periodic grid at the low corner (neighbours "
                         "only at +x, +y, +z: BASELINE config 3's 2x2x2 ranks all look like this)")
    a = ap.parse_args()
    import torch
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    rows = []
    for nz in a.nz:
        for k in a.k:
            s = Settings(L=a.L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                         noise=0.1, backend="AMDGPU")
            sim = GrayScott(s, init_domain((a.L, a.L, nz), 1, 0), fuse=k)
            sim.init_fields()
            lib, h = sim.engine.lib, sim.engine.h

            sides = 2 | 8 if a.one_sided else 15

            def run(z0, n0, z1, n1, tiles=0):
                native.check(lib, lib.gs_fused_runs_raw(h, k, z0, n0, z1, n1, tiles,
                                                        sides if tiles else 0), "fused_runs")

            def timed(*runs):
                for _ in range(3):
                    for r in runs:
                        run(*r)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.reps):
                    for r in runs:
                        run(*r)
                e1.record()
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / a.reps * 1e3  # us

            full = timed((0, nz, 0, 0))
            if a.packed and a.one_sided:
                ins = [(0, nz - k, 0, 0, 1)]
                shs = [(nz - k, k, 0, 0), (0, nz - k, 0, 0, 2)]
            elif a.packed:
                ins = [(k, nz - 2 * k, 0, 0, 1)]
                shs = [(0, k, nz - k, k), (k, nz - 2 * k, 0, 0, 2)]
            else:
                ins = [(k, nz - 2 * k, 0, 0)]
                shs = [(0, k, nz - k, k)]
            inner = timed(*ins)
            shell = timed(*shs)
            both = timed(*(ins + shs))
            row = {"local": [a.L, a.L, nz], "k": k, "packed": a.packed,
                   "one_sided": a.one_sided, "full_us": round(full, 1),
                   "inner_us": round(inner, 1), "shell_us": round(shell, 1),
                   "inner_plus_shell_us": round(both, 1),
                   "full_mlups": round(a.L * a.L * nz * k / full, 0),
                   "tile": sim.fused_choice().get(k)}
            rows.append(row)
            print(json.dumps(row), flush=True)
            sim.close()
            del sim
            torch.cuda.empty_cache()
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
