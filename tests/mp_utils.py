"""Multi-process harness: run N ranks over a gloo rendezvous on 127.0.0.1 and collect fields.

Mirrors the reference's functional `mpirun -n 4` tests (test/functional/functional-GrayScott.jl)
without MPI: one Python process per rank, torch.distributed gloo control plane.
"""
from __future__ import annotations

import os
import socket
import sys
import tempfile
import traceback

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, outdir, cfg):
    try:
        sys.path.insert(0, ROOT)
        os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": "0",
                           "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port),
                           "OMP_NUM_THREADS": "1"})
        os.environ.update(cfg.get("env") or {})
        from grayscott_amd.models.grayscott import GrayScott
        from grayscott_amd.parallel import dist as gdist
        from grayscott_amd.parallel.decomp import choose_dims, init_domain
        from grayscott_amd.utils.config import Settings

        from grayscott_amd.ops import native
        for name, value in (cfg.get("knobs") or {}).items():  # native test switches (gs/debug.h)
            native.debug_set(name, value, "hip")
        settings = Settings(**cfg["settings"])
        backend = "hip" if settings.backend.lower() in ("amdgpu", "hip", "gpu") else "cpu"
        ctx = gdist.init_from_env(backend)
        dims = cfg.get("dims") or choose_dims(settings.L, world, settings.decomposition, backend)
        dom = init_domain(settings.L, world, rank, periodic=settings.periodic, dims=dims)
        sim = GrayScott(settings, dom, ctx, fuse=cfg.get("fuse"), transport=cfg.get("transport"),
                        use_fused=cfg.get("use_fused", True))
        sim.init_fields()
        if cfg.get("random_init") is not None:
            sim.randomize_fields(seed=cfg["random_init"])
        if cfg.get("poison"):
            sim.poison_ghosts()
        sim.iterate(cfg["steps"])
        u, v = sim.get_fields()
        import json
        # per-phase timing of a further window (after the fields were taken)
        prof = sim.phase_profile(cfg["profile_steps"]) if cfg.get("profile_steps") else None
        info = json.dumps(sim.device_info())
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), u=u, v=v, info=info,
                 offsets=np.array(dom.proc_offsets), sizes=np.array(dom.proc_sizes),
                 step=sim.step, transport=sim.transport, overlapped=sim.overlapped,
                 gated=sim.gated, gate=json.dumps(sim.engine.gate_info(sim.engine.depth())),
                 profile=json.dumps(prof),
                 zplanes=sim.engine.plan()["zplanes"])
        sim.close()
        ctx.barrier()
        ctx.finalize()
    except Exception:
        with open(os.path.join(outdir, f"error{rank}.txt"), "w") as fh:
            fh.write(traceback.format_exc())
        raise


def run_ranks(world: int, cfg: dict, timeout: float = 240.0):
    """Run `world` ranks; return assembled global (u, v) as (Lz, Ly, Lx) arrays and metadata."""
    port = free_port()
    with tempfile.TemporaryDirectory() as outdir:
        ctx = mp.start_processes(_worker, args=(world, port, outdir, cfg), nprocs=world,
                                 join=False, start_method="spawn")
        # bounded: ranks still running after 3 x timeout are killed and the test fails (a hung
        # rank must end the test, not the GPU-test run).  join() returns False each time one
        # rank of several exits, so it is called until all have or the time is up
        import time
        deadline = time.monotonic() + 3 * timeout
        ok = ctx.join(timeout)
        while not ok and time.monotonic() < deadline:
            ok = ctx.join(max(1.0, deadline - time.monotonic()))
        if not ok:
            for p in ctx.processes:
                if p.is_alive():
                    p.kill()
            raise RuntimeError(f"{world} ranks did not finish within {3 * timeout:g} s")
        errs = [f for f in os.listdir(outdir) if f.startswith("error")]
        if errs:
            raise RuntimeError(open(os.path.join(outdir, errs[0])).read())
        L = cfg["settings"]["L"]
        Ls = (L, L, L) if isinstance(L, int) else L
        u = np.full((Ls[2], Ls[1], Ls[0]), np.nan)
        v = np.full_like(u, np.nan)
        meta = []
        for r in range(world):
            d = np.load(os.path.join(outdir, f"rank{r}.npz"))
            o, s = d["offsets"], d["sizes"]
            sl = (slice(o[2], o[2] + s[2]), slice(o[1], o[1] + s[1]), slice(o[0], o[0] + s[0]))
            u[sl] = d["u"]
            v[sl] = d["v"]
            meta.append({"step": int(d["step"]), "transport": str(d["transport"]),
                         "overlapped": bool(d["overlapped"]), "zplanes": bool(d["zplanes"]),
                         "gated": bool(d["gated"]), "gate": __import__("json").loads(str(d["gate"])),
                         "info": __import__("json").loads(str(d["info"])),
                         "profile": __import__("json").loads(str(d["profile"]))})
        return u, v, meta
