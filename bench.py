#!/usr/bin/env python3
"""Headline benchmark: MLUPS (cell updates / s, whole job) of the 3D Gray-Scott step.

BASELINE.json metric: "MLUPS (cell-updates/sec, whole node) at L=512 fp32, 1/2/4/8 MI355X".
Config: the reference example physics (examples/settings-files.toml: F=0.02, k=0.048, dt=1,
Du=0.2, Dv=0.1, noise=0.1) on an L^3 = 512^3 fp32 grid, decomposed over the N GPUs with the
reference's Dims_create factorisation (2 -> 2x1x1, 4 -> 2x2x1, 8 -> 2x2x2).  The global grid is
fixed as N grows (strong scaling).  Every timed step is a full update of all L^3 cells
including the Philox noise and the RCCL halo exchange.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--L 512] [--precision Float32]
  torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def distributed_selfcheck(ctx, backend, dims, fuse, transport, overlap, L=64, steps=9):
    """Before timing a multi-rank run, check the exact data path it will use (decomposition,
    transport, in-place halos, overlap, fuse depth) on a small grid against the numpy/torch
    golden model computed by every rank.  Returns (ok, max_abs_err, transport)."""
    import numpy as np

    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import reference as ref
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    L = max(L, 8 * max(dims))
    s = Settings(L=L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend="AMDGPU" if backend == "hip" else "CPU", seed=77, transport=transport,
                 overlap=overlap)
    dom = init_domain(L, ctx.world_size, ctx.rank, periodic=False, dims=dims)
    sim = GrayScott(s, dom, ctx, fuse=min(fuse, min(dom.proc_sizes)))
    try:
        sim.init_fields()
        sim.iterate(steps)
        u, v = sim.get_fields()
        used = sim.transport
    finally:
        sim.close()
    ru, rv = ref.run(L, steps, noise_amp=0.1, seed=77, dtype=np.float32, backend="torch")
    (ox, oy, oz), (nx, ny, nz) = dom.proc_offsets, dom.proc_sizes
    blk = (slice(oz, oz + nz), slice(oy, oy + ny), slice(ox, ox + nx))
    err = float(max(np.abs(u - ru[blk]).max(), np.abs(v - rv[blk]).max()))
    err = ctx.allreduce(err, "max")
    return err < 1e-4, err, used


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=40)
    ap.add_argument("--L", type=int, default=512)
    ap.add_argument("--precision", default="Float32")
    ap.add_argument("--fuse", type=int, default=0, help="steps per halo exchange (0 = auto)")
    ap.add_argument("--transport", default="auto")
    ap.add_argument("--no-fused-kernel", action="store_true")
    ap.add_argument("--noise", type=float, default=0.1)
    ap.add_argument("--backend", default="AMDGPU")
    ap.add_argument("--decomposition", default="auto", help="auto | balanced | z")
    ap.add_argument("--overlap", default="auto", help="auto | on | off")
    ap.add_argument("--init", default="random", choices=["random", "seed"],
                    help="random: u, v ~ U[0,1) (BASELINE.json); seed: the reference's seed cube")
    args = ap.parse_args(argv)

    import torch

    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import choose_dims, init_domain
    from grayscott_amd.parallel.dist import init_from_env
    from grayscott_amd.utils.config import Settings, load_backend_and_lang

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            print(f"bench.py: --gpus {args.gpus} needs a torchrun launch with "
                  f"--nproc-per-node {args.gpus}", file=sys.stderr)
            return 2
    settings = Settings(L=args.L, steps=args.steps, plotgap=args.steps + args.warmup + 1,
                        F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=args.noise,
                        precision=args.precision, backend=args.backend, fuse_steps=args.fuse,
                        transport=args.transport, decomposition=args.decomposition,
                        overlap=args.overlap)
    backend, _ = load_backend_and_lang(settings)
    ctx = init_from_env("hip" if backend == "hip" else "cpu")
    dims = choose_dims(args.L, ctx.world_size, args.decomposition, backend)
    dom = init_domain(args.L, ctx.world_size, ctx.rank, periodic=False, dims=dims)
    selfcheck = None
    if ctx.world_size > 1:
        # verify the multi-rank data path first; fall back to safer paths if it is wrong
        from grayscott_amd.models.grayscott import default_fuse
        fuse0 = args.fuse if args.fuse > 0 else default_fuse(backend, dom, settings.dtype_name)
        attempts = [(args.transport, args.overlap, None), (args.transport, "off", "0"),
                    ("torch", "off", "0")]
        for tr, ov, inplace in attempts:
            if inplace is not None:
                os.environ["GS_INPLACE_HALO"] = inplace
            ok, err, used = distributed_selfcheck(ctx, backend, dims, fuse0, tr, ov)
            selfcheck = {"ok": ok, "max_abs_err": err, "transport": used, "overlap": ov,
                         "inplace_halos": inplace is None}
            if ok:
                settings.transport, settings.overlap = tr, ov
                break
            if ctx.rank == 0:
                print(f"bench.py: multi-rank self-check FAILED ({selfcheck}); trying a safer "
                      f"data path", file=sys.stderr)
    sim = GrayScott(settings, dom, ctx, use_fused=not args.no_fused_kernel)
    sim.init_fields()
    if args.init == "random":
        sim.randomize_fields(seed=2024)

    def sync():
        sim.synchronize()
        if backend == "hip":
            torch.cuda.synchronize()

    sim.iterate(args.warmup)
    sync()
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    sim.iterate(args.steps)
    sync()
    t1 = time.perf_counter()
    ctx.barrier()
    local = t1 - t0
    elapsed = ctx.allreduce(local, "max")
    stats = sim.global_stats()
    cells = float(args.L) ** 3
    mlups = cells * args.steps / elapsed / 1e6
    if ctx.rank == 0:
        dims = "x".join(str(d) for d in dom.dims)
        rec = {
            "metric": f"MLUPS (cell-updates/sec, whole node) at L={args.L} "
                      f"{'fp32' if settings.dtype_name == 'float32' else 'fp64'}",
            "value": round(mlups, 1),
            "unit": "MLUPS",
            "n_gpus": ctx.world_size if backend == "hip" else 0,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 5),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32" if settings.dtype_name == "float32" else "fp64",
            "data": ("synthetic: random-init u, v ~ U[0,1) on device" if args.init == "random"
                     else "synthetic: reference seed-cube init") +
                    " + in-kernel Philox noise, examples/settings-files.toml physics",
            "config": {
                "model": "gray-scott-3d-7pt",
                "L": args.L,
                "global_batch": 1,
                "seq_len": args.L,
                "parallelism": (f"spatial-z-slabs {dims} ({sim.transport} plane halos, overlapped)"
                                if sim.overlapped else f"spatial-3d {dims}"),
                "dims": dom.dims,
                "local_extent": dom.proc_sizes,
                "fuse_steps": sim.fuse,
                "fused_kernel": {str(n): {"tile": c[0] or "default", "sched": c[1]}
                                 for n, c in sim.fused_choice().items()},
                "transport": sim.transport,
                "overlap": sim.overlapped,
                "noise": args.noise,
                "backend": backend,
            },
            "selfcheck": selfcheck,
            "check": {"mean_u": stats["mean_u"], "mean_v": stats["mean_v"],
                      "finite": all(map(lambda x: x == x, stats.values()))},
        }
        print(json.dumps(rec), flush=True)
    sim.close()
    ctx.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
