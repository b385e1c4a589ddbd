"""Application driver: the Gray-Scott time loop (reference src/GrayScott.jl).

Parity:
  * ``main(args)``      -- GrayScott.jl:68-103: settings -> init -> output stream -> loop
                           {iterate!, step += 1, write every plotgap} -> close -> finalize
  * ``julia_main()``    -- GrayScott.jl:40-48: catches errors, prints them, returns 1
  * verbose line        -- GrayScott.jl:88-91 ("Simulation at step s writing output step s/plotgap",
                           float division)
  * no output at step 0; `steps` steps; output steps plotgap, 2*plotgap, ...

Additions: checkpoint every ``checkpoint_freq`` steps and restart from ``restart_input`` (the
reference parses these keys but ignores them, D6), a JSON-lines perf log, optional global
diagnostics, and fault injection for restart testing (``GS_FAIL_AT_STEP=<n>`` makes every
rank exit with status 3 right after step n has been computed and checkpointed;
``GS_RAISE_AT_STEP=<n>`` with ``GS_FAIL_RANK=<r>`` makes rank r alone raise an error there).

Job-wide failure handling: the reference's julia_main catches, prints and
returns 1 (GrayScott.jl:40-48), and an MPI error aborts the whole job.  Here a rank that fails
in a multi-rank job aborts its RCCL communicator and exits at once (``os._exit(1)``, no
clean-up that could block on a collective), so its peers see the broken connection (gloo) or
the aborted communicator (RCCL watchdog) and fail too instead of waiting; every gloo
collective is also bounded by GS_COMM_TIMEOUT (parallel/dist.py).  Checkpoints
are written behind the simulation by default (``async_checkpoint``, io/checkpoint.py
``CheckpointWriter``): the data write runs on a host thread from the same snapshot as the output
step, and is committed before the next snapshot, at the end, or before a fault-injected exit.

The loop advances in chunks up to the next output/checkpoint event, so steps between events
run back to back in the native engine (temporal blocking, no per-step Python).
"""
from __future__ import annotations

import os
import sys
import time
import traceback
from typing import Optional, Sequence

from .io.checkpoint import restart as do_restart
from .io.checkpoint import CheckpointWriter, write_checkpoint
from .io.output import SimulationOutput
from .models.grayscott import GrayScott
from .parallel.decomp import choose_dims, init_domain
from .parallel.dist import init_from_env
from .utils.config import Settings, get_settings, load_backend_and_lang
from .utils.timers import DeviceTimer, PerfLog, PhaseTimer


def initialization(args: Sequence[str]):
    """communication.jl:15-33: settings, process group, decomposition, fields."""
    settings = get_settings(args)
    return initialize_from_settings(settings)


def initialize_from_settings(settings: Settings):
    backend, _ = load_backend_and_lang(settings)
    ctx = init_from_env(backend)
    if str(settings.decomposition).lower() == "tune":
        # time the candidate data paths on this node first (parallel/autotune.py)
        from .parallel.autotune import tune_data_path
        if ctx.world_size > 1 and not settings.periodic and isinstance(settings.L, int):
            t = tune_data_path(settings, ctx, settings.L, backend)
            settings.fuse_steps = t["fuse"]
            settings.transport, settings.overlap = t["transport"], t["overlap"]
            os.environ.update(t["env"])
            dims = t["dims"]
        else:
            dims = choose_dims(settings.L, ctx.world_size, "auto", backend)
    else:
        dims = choose_dims(settings.L, ctx.world_size, settings.decomposition, backend)
    domain = init_domain(settings.L, ctx.world_size, ctx.rank, periodic=settings.periodic,
                         dims=dims)
    sim = GrayScott(settings, domain, ctx)
    sim.init_fields()
    return ctx, settings, domain, sim


def _next_event(step: int, settings: Settings) -> int:
    nxt = settings.steps
    if settings.plotgap > 0:
        nxt = min(nxt, (step // settings.plotgap + 1) * settings.plotgap)
    if settings.checkpoint and settings.checkpoint_freq > 0:
        nxt = min(nxt, (step // settings.checkpoint_freq + 1) * settings.checkpoint_freq)
    return nxt


def run(settings: Settings, out=sys.stdout) -> dict:
    ctx, settings, domain, sim = initialize_from_settings(settings)
    rank = ctx.rank
    timer = PhaseTimer(sync=sim.synchronize)  # host phases: output, checkpoint, restart
    # compute intervals: timing events in stream order, nothing synchronised around them
    dtimer = DeviceTimer(sim.device if sim.backend == "hip" else None)
    perf = PerfLog(settings.perf_log, enabled=(rank == 0))
    fail_at = int(os.environ.get("GS_FAIL_AT_STEP", "-1"))
    raise_at = int(os.environ.get("GS_RAISE_AT_STEP", "-1"))
    fail_rank = int(os.environ.get("GS_FAIL_RANK", "-1"))
    step = 0
    if settings.restart:
        with timer.phase("restart"):
            step = do_restart(sim, settings, ctx)
        if rank == 0 and settings.verbose:
            print(f"Restarting from step {step} ({settings.restart_input})", file=out, flush=True)
    with timer.phase("io_init"):
        # a restarted run continues the existing output: its steps up to the restart step stay
        stream = SimulationOutput(settings, domain, ctx,
                                  append_after_step=step if settings.restart else None)
        if settings.plotgap > 0:
            stream.prepare(sim)
    if (settings.restart and settings.plotgap > 0 and step > 0 and step % settings.plotgap == 0
            and stream.last_step != step):
        # the failed run had not committed this output step: the restored state is that step's
        # state bit for bit (Philox keyed on global cell and step), so write it now
        with timer.phase("output"):
            stream.write_step(step, sim)
    first_step = step
    ckpt_on = settings.checkpoint and settings.checkpoint_freq > 0
    ckpt = (CheckpointWriter(settings, domain, ctx)
            if ckpt_on and getattr(settings, "async_checkpoint", True) else None)
    t_loop = time.perf_counter()
    cells = float(domain.L[0]) * domain.L[1] * domain.L[2]

    def log_compute(wait: bool = False) -> None:
        for sec, m in dtimer.completed(wait=wait):
            perf.write(step=m["step"], steps=m["steps"], compute_s=sec, io_s=m["io_s"],
                       mlups=cells * m["steps"] / max(sec, 1e-12) / 1e6, ranks=ctx.world_size)

    while step < settings.steps:
        nxt = _next_event(step, settings)
        tok = dtimer.start()
        sim.iterate(nxt - step)
        nsteps = nxt - step
        meta = {"step": nxt, "steps": nsteps, "io_s": 0.0}
        dtimer.stop(tok, meta)
        step = nxt
        io_s = 0.0
        do_out = settings.plotgap > 0 and step % settings.plotgap == 0
        do_ckpt = ckpt_on and step % settings.checkpoint_freq == 0
        if ckpt is not None and ckpt.pending and (do_out or do_ckpt):
            # the previous checkpoint's data thread reads the snapshot buffers: commit it
            # before they are reused
            t1 = time.perf_counter()
            with timer.phase("checkpoint"):
                ckpt.finish()
            io_s += time.perf_counter() - t1
        snap = None
        if do_out:
            if rank == 0 and settings.verbose:
                print(f"Simulation at step {step} writing output step "
                      f"{step / settings.plotgap}", file=out, flush=True)
            t1 = time.perf_counter()
            with timer.phase("output", sync=not stream.async_io):
                snap = stream.write_step(step, sim)
            io_s += time.perf_counter() - t1
            if settings.diagnostics:
                d = sim.global_stats()
                if rank == 0:
                    print(f"  step {step}: " + " ".join(f"{k}={v:.6g}" for k, v in d.items()),
                          file=out, flush=True)
        if do_ckpt:
            t1 = time.perf_counter()
            with timer.phase("checkpoint"):
                # output steps before the checkpoint's are committed first (output_queue > 1
                # keeps several in flight): a restart from it rewrites only its own step
                stream.commit_through(step - 1)
                if ckpt is not None:
                    ckpt.start(step, sim, snap)
                else:
                    write_checkpoint(settings.checkpoint_output, step, sim, settings, ctx)
            io_s += time.perf_counter() - t1
        meta["io_s"] = io_s  # the interval's record is written once its events have completed
        log_compute()
        if raise_at >= 0 and step >= raise_at and fail_rank in (-1, rank):
            raise RuntimeError(f"injected failure on rank {rank} at step {step} "
                               "(GS_RAISE_AT_STEP)")
        if fail_at >= 0 and step >= fail_at:
            if ckpt is not None:
                ckpt.finish()
            sys.stdout.flush()
            os._exit(3)  # simulated node failure (no clean shutdown)
    if ckpt is not None and ckpt.pending:
        with timer.phase("checkpoint"):
            ckpt.finish()
    sim.synchronize()
    loop_s = time.perf_counter() - t_loop
    log_compute(wait=True)
    compute_s = dtimer.total
    with timer.phase("io_close"):
        stream.close()
    result = {"steps": step, "loop_s": loop_s, "compute_s": compute_s,
              "mlups_compute": cells * (step - first_step) / max(compute_s, 1e-12) / 1e6,
              "timers": {**timer.summary(),
                         "compute": {"seconds": compute_s, "calls": dtimer.count,
                                     "clock": "device events" if dtimer.device is not None
                                     else "host"}},
              "ranks": ctx.world_size, "fuse": sim.depth,
              "transport": sim.transport}
    perf.write(summary=result)
    perf.close()
    sim.close()
    ctx.finalize()
    return result


def main(args: Optional[Sequence[str]] = None) -> dict:
    """GrayScott.main (GrayScott.jl:68-103)."""
    settings = get_settings(list(sys.argv[1:] if args is None else args))
    return run(settings)


def abort_job(code: int = 1) -> None:
    """End this rank of a multi-rank job now: abort the RCCL communicator (peers blocked in a
    halo exchange get an error) and exit without interpreter clean-up (which could block in a
    collective).  Never returns."""
    try:
        from .ops import native
        native.rccl_abort()
    except Exception:
        pass
    try:
        sys.stdout.flush()
        sys.stderr.flush()
    finally:
        os._exit(code)


def julia_main(args: Optional[Sequence[str]] = None) -> int:
    """GrayScott.julia_main (GrayScott.jl:40-48): 0 on success, 1 on error.  In a multi-rank
    job an error ends this rank at once (``abort_job``) so the job fails fast."""
    from .parallel.launch import launcher_env
    try:
        main(args)
    except SystemExit as e:
        return int(e.code or 0)
    except BaseException:
        traceback.print_exc()
        if launcher_env()[1] > 1:
            rank = launcher_env()[0]
            print(f"rank {rank}: aborting the job", file=sys.stderr, flush=True)
            abort_job(1)
        return 1
    return 0
