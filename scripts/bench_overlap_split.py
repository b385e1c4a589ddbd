#!/usr/bin/env python3
"""Kernel-side cost of the comm/compute-overlap split on ONE MI355X (no communication).

For a sub-domain (what one rank of an N-GPU run owns) it times, per k-step pass:
  full   -- one fused launch over the whole interior (the non-overlapped pass),
  inner  -- the launch that runs while the halos are in flight: all x-y tiles over the planes
            at least k from a z face with a neighbour, outputs clipped to at least k from every
            x / y face with one (cell-granular store mask), workgroup slots left free,
  shell  -- the k-deep face slabs after the halos land (engine.h shell_run: k_slab, or the
            z slabs through k_fused -- the faster of the two, chosen at first use).
The overlapped pass costs shell + max(inner, exchange); the plain one full + exchange.
Default: a z slab (neighbours at -z and +z).  --packed: one rank of the balanced grid with
neighbours on every side; --one-sided: neighbours only at +x, +y, +z (BASELINE config 3's
2x2x2 ranks all look like this).

  python scripts/bench_overlap_split.py --nz 64 128 256 --k 2 3
  python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 3
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

            if a.packed and a.one_sided:
                sides = 2 | 8 | 32
            elif a.packed:
                sides = 63
            else:
                sides = 16 | 32
            z0 = k if sides & 16 else 0
            z1 = nz - k if sides & 32 else nz

            def run(kind):
                if kind == "full":
                    rc = lib.gs_fused_runs_raw(h, k, 0, nz, 0, 0, 0, 0)
                elif kind == "inner":
                    rc = lib.gs_fused_runs_raw(h, k, z0, z1 - z0, 0, 0, sides & 15, 1)
                elif kind == "shell":
                    rc = lib.gs_shell_raw(h, k, sides, -1)
                else:  # ("faces", subset of sides, variant)
                    rc = lib.gs_shell_raw(h, k, kind[1], kind[2])
                native.check(lib, rc, str(kind))

            def timed(*runs):
                for _ in range(3):
                    for r in runs:
                        run(r)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for _ in range(a.reps):
                    for r in runs:
                        run(r)
                e1.record()
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / a.reps * 1e3  # us

            full = timed("full")
            ins, shs = ["inner"], ["shell"]
            inner = timed(*ins)
            shell = timed(*shs)
            both = timed(*(ins + shs))
            # per face group: z slabs through k_slab (v0) or k_fused (v1), x and y slabs
            faces = {}
            for name, bits in (("z", sides & 48), ("x", sides & 3), ("y", sides & 12)):
                if bits:
                    for v in ((0, 1) if name == "z" else (0,)):
                        faces[f"{name}_v{v}_us"] = round(timed(("faces", bits, v)), 1)
            # the whole shell through each variant
            if (sides & 48) and (sides & 15):
                for v in (0, 1):
                    faces[f"all_v{v}_us"] = round(timed(("faces", sides, v)), 1)
            row = {"local": [a.L, a.L, nz], "k": k, "packed": a.packed, "faces": faces,
                   "one_sided": a.one_sided, "full_us": round(full, 1),
                   "inner_us": round(inner, 1), "shell_us": round(shell, 1),
                   "inner_plus_shell_us": round(both, 1),
                   "full_mlups": round(a.L * a.L * nz * k / full, 0),
                   "sides": sides, "tile": sim.fused_choice().get(k)}
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
