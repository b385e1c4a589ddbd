#!/usr/bin/env python3
"""Headline benchmark: MLUPS (cell updates / s, whole job) of the 3D Gray-Scott step.

BASELINE.json metric: "MLUPS (cell-updates/sec, whole node) at L=512 fp32, 1/2/4/8 MI355X".
Config: the reference example physics (examples/settings-files.toml: F=0.02, k=0.048, dt=1,
Du=0.2, Dv=0.1, noise=0.1) on an L^3 = 512^3 fp32 grid, decomposed over the N GPUs (z slabs
1x1xN or the reference's Dims_create grid 2x2x2, whichever runs faster here).  The global grid
is fixed as N grows (strong scaling).  Every timed step is a full update of all L^3 cells
including the Philox noise and the RCCL halo exchange.  With N > 1 the multi-rank data path
(z slabs or the balanced grid, fuse depth, transport) is verified against the golden model and
then picked by a short timed run of each candidate before the timed region.

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
    tuning = None
    if ctx.world_size > 1:
        # Verify every candidate multi-rank data path against the golden model, then time a
        # short run of each on this problem and keep the fastest (parallel/autotune.py): the
        # z-slab vs balanced trade-off depends on this node's xGMI / RCCL rates.
        from grayscott_amd.parallel.autotune import tune_data_path
        cands = None
        if args.decomposition != "auto" or args.fuse > 0:
            cands = [(dims, args.fuse)]
        log = (lambda m: print(f"bench.py: {m}", file=sys.stderr, flush=True))
        tuning = tune_data_path(settings, ctx, args.L, backend, cands=cands, log=log)
        dims = tuning["dims"]
        settings.fuse_steps = tuning["fuse"]
        settings.transport, settings.overlap = tuning["transport"], tuning["overlap"]
        os.environ.update(tuning["env"])
    dom = init_domain(args.L, ctx.world_size, ctx.rank, periodic=False, dims=dims)
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
            "data_path_tuning": tuning and tuning["table"],
            "check": {"mean_u": stats["mean_u"], "mean_v": stats["mean_v"],
                      "finite": all(map(lambda x: x == x, stats.values()))},
        }
        print(json.dumps(rec), flush=True)
    sim.close()
    ctx.finalize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
