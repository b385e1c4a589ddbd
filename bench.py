#!/usr/bin/env python3
"""Headline benchmark: MLUPS (cell updates / s, whole job) of the 3D Gray-Scott step.

BASELINE.json metric: "MLUPS (cell-updates/sec, whole node) at L=512 fp32, 1/2/4/8 MI355X".
Config: the reference example physics (examples/settings-files.toml: F=0.02, k=0.048, dt=1,
Du=0.2, Dv=0.1, noise=0.1) on an L^3 = 512^3 fp32 grid with random-init u, v, decomposed over
the N GPUs.  The global grid is fixed as N grows (strong scaling).  Every timed step is a full
update of all L^3 cells including the Philox noise and the RCCL halo exchange.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--L 512] [--precision Float32]
  torchrun --nproc-per-node N bench.py --gpus N ...       (or mpiexec / srun)

``--gpus N`` without a launcher starts the N ranks itself (parallel/launch.py: one worker
process per GPU over a 127.0.0.1 rendezvous; this parent never touches the GPU) and exits with
the job's status.  Rank 0 prints ONE JSON line.

Checks of the timed path:
  * any N, after the timed region: the state is reset to the benchmark's initial state (the
    random init is a function of the global cell, so every rank regenerates its block), the
    timed configuration -- decomposition, transport, overlap, fuse depth, precision, size --
    runs ``--check-steps`` steps, and each rank compares its block with the native OpenMP
    golden model run on that block grown by the same number of cells on every side with a
    neighbour (the cone the steps depend on): ``check.max_abs_err`` over all ranks (a failure
    makes the run exit non-zero);
  * N > 1 (before timing): every candidate data path (z slabs / the reference's Dims_create
    grid, overlap, transport) is checked against the golden model on a small grid and timed on
    the real problem (parallel/autotune.py); the fastest one is used, and the reference grid's
    own timing is reported (``reference_grid``; ``config3_2x2x2`` at N = 8, BASELINE config 3).
The JSON also records what RCCL saw: communicator size and each rank's device and PCI bus id.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

T_START = time.perf_counter()
_JSON_FD = 1  # the original stdout (main() points fd 1 at stderr for the run)
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# What a failure record can report: the phase the run is in and the data-path tuning rows
# finished so far (rank 0).  One JSON line per job, whatever happens (_emit_once).
_PROGRESS = {"phase": "start", "rows": []}
_EMIT = threading.Lock()
_EMITTED = [False, True]  # printed, and whether that line reported success


def parse_args(argv):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=None)
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
    ap.add_argument("--check", default="auto", choices=["auto", "golden", "none"],
                    help="golden-model check of the timed path (auto: 1 rank, HIP)")
    ap.add_argument("--check-steps", type=int, default=6)
    ap.add_argument("--profile-passes", type=int, default=10,
                    help="passes of the per-phase timing window run after the timed region "
                         "(0 = off)")
    ap.add_argument("--tune-budget", type=float, default=float(os.environ.get("GS_TUNE_BUDGET_S",
                                                                                "180")),
                    help="seconds for the multi-rank data-path tuning (checks + timing)")
    ap.add_argument("--deadline", type=float,
                    default=float(os.environ.get("GS_BENCH_DEADLINE_S", "540")),
                    help="seconds from start after which every rank gives up: rank 0 prints a "
                         "JSON line with status 'timeout' (the phase it was in, the tuning rows "
                         "finished) and the job exits 124 (0 = off)")
    ap.add_argument("--debug-knob", action="append", default=[], metavar="NAME=VALUE",
                    help="set a native test switch on every rank (csrc/include/gs/debug.h; "
                         "rehearsals on one GPU, e.g. gated=2)")
    ap.add_argument("--timeout", type=float, default=0.0,
                    help="self-launched jobs: kill all ranks after this many seconds (default: "
                         "the deadline + 60 s)")
    return ap.parse_args(argv)


def _metric_name(args) -> str:
    return (f"MLUPS (cell-updates/sec, whole node) at L={args.L} "
            f"{'fp32' if args.precision.lower() in ('float32', 'fp32') else 'fp64'}")


def failure_record(args, status: str, n_gpus: int, **extra) -> dict:
    """The one JSON line of a job that produced no measurement: the contract's keys with
    ``value`` null, ``status`` ("timeout", "rank_failed", "error"), the phase the job was in
    and the data-path tuning rows it finished."""
    fp32 = args.precision.lower() in ("float32", "fp32")
    rec = {"metric": _metric_name(args), "value": None, "unit": "MLUPS", "n_gpus": n_gpus,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": None,
           "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
           "dtype": "fp32" if fp32 else "fp64",
           "data": "synthetic: random-init u, v ~ U[0,1) on device" if args.init == "random"
                   else "synthetic: reference seed-cube init",
           "config": {"model": "gray-scott-3d-7pt", "L": args.L, "global_batch": 1,
                      "seq_len": args.L, "parallelism": f"spatial-3d ({n_gpus} ranks)"},
           "status": status, "phase": _PROGRESS["phase"],
           "data_path_tuning": list(_PROGRESS["rows"]),
           # what the ranks measured of their links before the failure (first contact on a
           # node: the probe runs before any candidate; None if it did not get that far)
           "link_probe": _PROGRESS.get("link_probe"),
           "wall_s": round(time.perf_counter() - T_START, 2)}
    rec.update(extra)
    return rec


def _emit_once(rec: dict) -> bool:
    """Write the job's JSON line (at most once per process)."""
    with _EMIT:
        if _EMITTED[0]:
            return False
        _EMITTED[0] = True
        _EMITTED[1] = rec.get("status") == "ok"
        os.write(_JSON_FD, (json.dumps(rec) + "\n").encode())
        return True


def _progress_row(row: dict) -> None:
    """A finished data-path tuning row (rank 0): kept for a failure record and appended to
    GS_BENCH_PROGRESS (set by a self-launching parent, which reports it if the job dies)."""
    _PROGRESS["rows"].append(row)
    path = os.environ.get("GS_BENCH_PROGRESS")
    if path:
        try:
            with open(path, "a") as f:
                f.write(json.dumps(row) + "\n")
        except OSError:
            pass


def _progress_link(link) -> None:
    """The link probe's result (rank 0) into GS_BENCH_PROGRESS too, so a self-launching parent
    can report it if the job dies later."""
    path = os.environ.get("GS_BENCH_PROGRESS")
    if path and link is not None:
        try:
            with open(path, "a") as f:
                f.write(json.dumps({"link_probe": link}) + "\n")
        except OSError:
            pass


def start_deadline(args, rank: int, world: int) -> None:
    """Every rank: once ``args.deadline`` seconds have passed since start, rank 0 prints the
    failure record (status "timeout") and every rank exits 124 at once -- a first-contact stall
    on a fresh node (RCCL bootstrap, a peer that never joins, a device wait) yields a
    parseable line inside the driver's own limit instead of nothing."""
    if not args.deadline or args.deadline <= 0:
        return

    def fire():
        left = args.deadline - (time.perf_counter() - T_START)
        if left > 0:
            time.sleep(left)
        if _EMITTED[0]:
            # the result line is out: only the teardown is left, give it a minute, then end
            # with the status of the line already printed
            time.sleep(60)
            os._exit(0 if _EMITTED[1] else 1)
        if rank == 0:
            _emit_once(failure_record(args, "timeout", world, deadline_s=args.deadline))
        print(f"bench.py: rank {rank}: deadline of {args.deadline:g} s reached in phase "
              f"{_PROGRESS['phase']!r}; exiting", file=sys.stderr, flush=True)
        sys.stderr.flush()
        os._exit(124)

    threading.Thread(target=fire, name="bench-deadline", daemon=True).start()


def self_launch(args, argv, ngpus: int) -> int:
    """``--gpus N`` without a launcher: run the N ranks here (parallel/launch.py), forward rank
    0's JSON line, and if the job ended without one (a rank failed, the job's time limit),
    print a failure record naming the failing rank and the tuning rows rank 0 streamed to
    GS_BENCH_PROGRESS."""
    import tempfile

    from grayscott_amd.parallel.launch import spawn_local

    timeout = args.timeout or ((args.deadline + 60.0) if args.deadline > 0 else None)
    with tempfile.TemporaryDirectory(prefix="gs_bench_") as tmp:
        out_path = os.path.join(tmp, "rank0.out")
        prog = os.path.join(tmp, "progress.jsonl")
        info: dict = {}
        with open(out_path, "w") as out0:
            rc = spawn_local(ngpus, [sys.executable, os.path.abspath(__file__)] + argv,
                             timeout=timeout, cwd=ROOT, rank0_stdout=out0, info=info,
                             extra_env={"GS_BENCH_PROGRESS": prog})
        with open(out_path) as f:
            text = f.read()
        lines = [l for l in text.splitlines() if l.startswith("{")]
        if lines:
            line = lines[-1]
            if rc != 0:
                try:
                    rec = json.loads(line)
                except ValueError:
                    rec = None
                if isinstance(rec, dict) and rec.get("value") is None:
                    # rank 0's own failure record: name the first rank this parent saw fail
                    # (a deadline stays a timeout: every rank exits 124 then, in any order)
                    if info.get("failed_rank") not in (None, 0) and rec.get("status") != "timeout":
                        rec["status"] = "rank_failed"
                    rec["failed_rank"] = info.get("failed_rank")
                    rec["exit_codes"] = info.get("codes")
                    line = json.dumps(rec)
            sys.stdout.write(line + "\n")
            sys.stdout.flush()
            return rc
        rows = []
        if os.path.exists(prog):
            with open(prog) as f:
                rows = [json.loads(l) for l in f if l.strip()]
        links = [r["link_probe"] for r in rows if "link_probe" in r]
        _PROGRESS["link_probe"] = links[-1] if links else None
        _PROGRESS["rows"] = [r for r in rows if "link_probe" not in r]
        _PROGRESS["phase"] = "unknown (no line from rank 0)"
        status = "timeout" if info.get("timed_out") else "rank_failed"
        rec = failure_record(args, status, ngpus, failed_rank=info.get("failed_rank"),
                             exit_codes=info.get("codes"))
        sys.stdout.write(json.dumps(rec) + "\n")
        sys.stdout.flush()
        return rc if rc else 1


def main(argv=None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    args = parse_args(argv)
    from grayscott_amd.parallel.launch import launcher_env

    rank, world, _ = launcher_env()
    ngpus = args.gpus if args.gpus is not None else world
    if ngpus > 1 and world == 1:
        # self-launch: one worker per GPU, before anything initialises HIP in this process
        return self_launch(args, argv, ngpus)
    # a blocked halo wait or control-plane collective becomes an error after this long (the
    # driver's own limit is minutes; a hung rank must not eat it)
    os.environ.setdefault("GS_COMM_TIMEOUT", "120")
    if ngpus != world:
        print(f"bench.py: --gpus {ngpus} but the launcher started {world} ranks", file=sys.stderr)
        return 2
    # stdout carries exactly one line, the JSON record: whatever the libraries print on fd 1
    # (RCCL's version banner, gloo's rendezvous report) goes to stderr instead
    global _JSON_FD
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)
    start_deadline(args, rank, world)
    try:
        return run(args)
    except BaseException as ex:
        if rank == 0 and not isinstance(ex, (KeyboardInterrupt, SystemExit)):
            # (with several ranks the cause may be a peer that failed first: a self-launching
            # parent adds the first failing rank it saw)
            _emit_once(failure_record(args, "error", world,
                                      error=f"rank 0: {type(ex).__name__}: {ex}"[:400]))
        if world > 1:
            # one failed rank ends the job now instead of leaving its peers blocked
            import traceback
            traceback.print_exc()
            from grayscott_amd.driver import abort_job
            abort_job(1)
        raise


def golden_check(sim, settings, dom, nsteps: int, init_seed):
    """Reset the (distributed) state to the benchmark's initial state, advance it ``nsteps``
    steps on the timed path, and compare this rank's block with the native OpenMP golden model
    (CPU backend, single-step kernel, same Philox stream) run on the block grown by ``nsteps``
    cells on every side with a neighbour: outside-in errors of the grown box's artificial
    boundary travel one cell per step, so the block itself is exact.  ``init_seed``: the random
    init's seed (None: the reference's seed cube).  Returns this rank's max |difference|."""
    import copy

    import numpy as np

    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import CartDomain
    from grayscott_amd.parallel.dist import DistContext

    sim.engine.init_fields()
    if init_seed is not None:
        sim.randomize_fields(seed=init_seed)
    sim.iterate(nsteps)
    ug, vg = sim.get_fields()
    lo, hi = [], []
    for a in range(3):
        o, n, L = dom.proc_offsets[a], dom.proc_sizes[a], dom.L[a]
        lo.append(max(0, o - nsteps))
        hi.append(min(L, o + n + nsteps))
    sub = CartDomain(nprocs=1, rank=0, L=tuple(dom.L), dims=[1, 1, 1], coords=(0, 0, 0),
                     proc_sizes=[h - l for l, h in zip(lo, hi)], proc_offsets=lo,
                     periodic=False, nbr27=[-1] * 27)
    cs = copy.copy(settings)
    cs.backend, cs.fuse_steps, cs.transport = "CPU", 1, "none"
    # the node's ranks run their golden models at once: each gets its share of the cores
    from grayscott_amd.ops import native
    local = int(os.environ.get("LOCAL_WORLD_SIZE", "0") or 0) or max(1, dom.nprocs)
    keep = native.cpu_threads()  # OMP_NUM_THREADS, or every core OpenMP sees
    cores = min(keep, len(os.sched_getaffinity(0)))
    native.cpu_threads(max(1, cores // local))
    cpu = GrayScott(cs, sub, DistContext())
    try:
        cpu.engine.init_fields()
        if init_seed is not None:
            cpu.randomize_fields(seed=init_seed)
        cpu.iterate(nsteps)
        uc, vc = cpu.get_fields()
    finally:
        cpu.close()
        native.cpu_threads(keep)
    (ox, oy, oz), (nx, ny, nz) = dom.proc_offsets, dom.proc_sizes
    blk = (slice(oz - lo[2], oz - lo[2] + nz), slice(oy - lo[1], oy - lo[1] + ny),
           slice(ox - lo[0], ox - lo[0] + nx))
    err = float(max(np.abs(ug - uc[blk]).max(), np.abs(vg - vc[blk]).max()))
    return err if err == err else float("inf")


def parallelism_label(dims, transport: str, overlapped: bool, gated: bool = False) -> str:
    """``spatial-z-slabs 1x1x8 (ipc plane halos, overlapped)``, ``spatial-3d 2x2x2 (rccl packed
    halos)``, ``spatial-3d 2x2x2 (ipc packed halos, gated)``, ``spatial-3d 1x1x1``: the process
    grid, and with neighbours the halo transport (z slabs exchange contiguous ghost planes in
    place, other grids packed faces / edges / corners) and whether the exchange overlaps the
    inner update -- gated: inside the pass's own fused launch (csrc/hip/gate.hpp)."""
    dstr = "x".join(str(int(d)) for d in dims)
    if all(int(d) == 1 for d in dims):
        return f"spatial-3d {dstr}"
    zslab = int(dims[0]) == 1 and int(dims[1]) == 1
    kind = "plane" if zslab else "packed"
    tail = ", gated" if gated else (", overlapped" if overlapped else "")
    return f"spatial-{'z-slabs' if zslab else '3d'} {dstr} ({transport} {kind} halos{tail})"


def profile_phases(sim, ctx, passes: int):
    """Per-phase device timing of ``passes`` passes of this data path, run after
    the timed region (csrc/include/gs/phase.h: hipEvents in stream order on the compute and
    communication streams).  Returns (on rank 0) ``{"per_rank": [...], "summary": {...}}``: the
    summary holds, per phase, the slowest rank's median microseconds per pass, and the slowest
    rank's pass time, exchange span and critical path; ``accounted`` is the smallest share of a
    rank's measured pass time that its parts explain."""
    prof = sim.phase_profile(passes * max(1, int(sim.depth)))
    return summarize_profiles(ctx.gather_object(prof))


def summarize_profiles(rows):
    """The ``phases`` entry from every rank's GrayScott.phase_profile (rank 0; None elsewhere)."""
    if not rows:
        return None
    names = sorted(set().union(*(r["phase_us"] for r in rows)))
    acc = [r["accounted"] for r in rows if r.get("accounted") is not None]
    gbs = [r["link_GBps"] for r in rows if r.get("link_GBps")]
    summary = {
        "passes": rows[0]["passes"], "steps_per_pass": rows[0]["depth"],
        "transport": rows[0]["transport"], "overlapped": rows[0]["overlapped"],
        "gated": rows[0].get("gated", False), "gate": rows[0].get("gate"),
        "chained": rows[0].get("chained", False),
        "pass_us": round(max(r["pass_us"] for r in rows), 2),
        "phase_us": {k: round(max(r["phase_us"].get(k, 0.0) for r in rows), 2) for k in names},
        "exchange_us": round(max(r["exchange_us"] for r in rows), 2),
        "critical_us": round(max(r["critical_us"] for r in rows), 2),
        "accounted": round(min(acc), 3) if acc else None,
        "bytes_per_neighbour_max": max((max(r["bytes_per_neighbour"].values(), default=0)
                                        for r in rows), default=0),
        "link_GBps_min": min(gbs) if gbs else None,
    }
    for r in rows:
        for k in ("window_us", "pass_us", "exchange_us", "critical_us"):
            r[k] = round(r[k], 2)
        r["phase_us"] = {k: round(v, 2) for k, v in r["phase_us"].items()}
    return {"summary": summary, "per_rank": rows}


def profile_reference_grid(settings, ctx, args, dims, row, passes: int):
    """profile_phases on the reference's Dims_create grid with the data path (fuse depth,
    transport, overlap, engine knobs) its best tuning row used."""
    import copy

    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.autotune import _env
    from grayscott_amd.parallel.decomp import init_domain

    s = copy.copy(settings)
    s.fuse_steps, s.transport, s.overlap = row["fuse"], row["transport"], row["overlap"]
    env = dict(row.get("env", {}))
    if not row.get("inplace_halos", True):
        env["GS_INPLACE_HALO"] = "0"
    sim, prof, err = None, None, None
    with _env(env):
        try:
            dom = init_domain(args.L, ctx.world_size, ctx.rank, periodic=False, dims=dims)
            sim = GrayScott(s, dom, ctx)
            sim.init_fields()
            sim.randomize_fields(seed=2024)
            sim.iterate(4 * max(1, int(sim.depth)))
            prof = sim.phase_profile(passes * max(1, int(sim.depth)))
        except Exception as ex:  # agreed below: a rank failing alone never strands the others
            err = f"rank {ctx.rank}: {type(ex).__name__}: {ex}"[:200]
        # every rank gets here whatever failed locally, and all agree before any collective
        # that needs every rank's result (the gather below, the IPC close barrier)
        ok = ctx.allreduce(0.0 if err else 1.0, "min") > 0
        if sim is not None:
            try:
                sim.synchronize()
            except Exception as ex:
                err = err or f"rank {ctx.rank}: {ex}"[:200]
        ctx.barrier()  # no rank frees buffers its peers may still write (IPC)
        if sim is not None:
            sim.close(barrier=False)
    if not ok:
        errs = [e for e in ctx.allgather_object(err) if e]
        return {"error": "; ".join(errs)[:400]} if ctx.rank == 0 else None
    out = summarize_profiles(ctx.gather_object(prof))
    if out is not None:
        out["summary"]["dims"] = list(dims)
    return out


def run(args) -> int:
    import torch

    if args.debug_knob and args.backend.lower() in ("amdgpu", "hip", "gpu"):
        from grayscott_amd.ops import native
        for kv in args.debug_knob:
            name, _, value = kv.partition("=")
            native.debug_set(name.strip(), float(value))

    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import choose_dims, dims_create, init_domain
    from grayscott_amd.parallel.dist import init_from_env
    from grayscott_amd.utils.config import Settings, load_backend_and_lang

    settings = Settings(L=args.L, steps=args.steps, plotgap=args.steps + args.warmup + 1,
                        F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=args.noise,
                        precision=args.precision, backend=args.backend, fuse_steps=args.fuse,
                        transport=args.transport, decomposition=args.decomposition,
                        overlap=args.overlap)
    backend, _ = load_backend_and_lang(settings)
    ctx = init_from_env("hip" if backend == "hip" else "cpu")
    dims = choose_dims(args.L, ctx.world_size, args.decomposition, backend)
    _PROGRESS["phase"] = "data-path tuning"
    tuning = None
    link = None
    t_tune = time.perf_counter()
    if ctx.world_size > 1 and backend == "hip" and os.environ.get("GS_LINK_PROBE", "1") != "0":
        # every pair of ranks measures its own link (IPC peer stores and RCCL send / receive at
        # the candidates' message sizes) before anything is timed: reported as link_probe, and
        # the tuner's model skips the candidates it says lose by > 20 % (parallel/linkprobe.py)
        _PROGRESS["phase"] = "link probe"
        from grayscott_amd.parallel.linkprobe import probe_links
        link = probe_links(ctx, log=lambda m: print(f"bench.py: {m}", file=sys.stderr,
                                                     flush=True))
        _PROGRESS["link_probe"] = link
        if ctx.rank == 0:
            _progress_link(link)
        if link and link.get("rccl_failed"):
            # the engines' "auto" transport chain starts after RCCL (agreed: same dict everywhere)
            from grayscott_amd.models import grayscott as _gsm
            _gsm._RCCL_FAILED[0] = True
        _PROGRESS["phase"] = "data-path tuning"
    if ctx.world_size > 1:
        # Verify every candidate multi-rank data path against the golden model, then time a
        # short run of each on this problem and keep the fastest (parallel/autotune.py): the
        # z-slab vs balanced trade-off depends on this node's xGMI / RCCL rates.
        from grayscott_amd.parallel.autotune import tune_data_path
        cands = None
        if args.decomposition != "auto" or args.fuse > 0:
            cands = [(dims, args.fuse)]
        log = (lambda m: print(f"bench.py: {m}", file=sys.stderr, flush=True))
        tuning = tune_data_path(settings, ctx, args.L, backend, cands=cands, log=log,
                                budget_s=args.tune_budget,
                                on_row=_progress_row if ctx.rank == 0 else None, link=link)
        dims = tuning["dims"]
        settings.fuse_steps = tuning["fuse"]
        settings.transport, settings.overlap = tuning["transport"], tuning["overlap"]
        os.environ.update(tuning["env"])
    tuning_s = time.perf_counter() - t_tune
    _PROGRESS["phase"] = "set-up of the chosen data path"
    dom = init_domain(args.L, ctx.world_size, ctx.rank, periodic=False, dims=dims)
    sim = GrayScott(settings, dom, ctx, use_fused=not args.no_fused_kernel)
    sim.init_fields()
    if args.init == "random":
        sim.randomize_fields(seed=2024)

    check = {}
    # the golden check of the timed path runs after timing (a seconds-long CPU golden run
    # before the timed region would leave the GPU idle right before it, and its clocks take
    # milliseconds to come back); the initial state is regenerated then
    do_golden = (args.check == "golden" or (args.check == "auto" and backend == "hip"))
    do_golden = do_golden and args.check_steps > 0

    def sync():
        sim.synchronize()
        if backend == "hip":
            torch.cuda.synchronize()

    _PROGRESS["phase"] = "warm-up"
    sim.iterate(args.warmup)
    sync()
    if int(os.environ.get("GS_FAIL_RANK", "-1")) in (-1, ctx.rank):
        if os.environ.get("GS_RAISE_AT_STEP") is not None:
            raise RuntimeError(f"injected failure on rank {ctx.rank} (GS_RAISE_AT_STEP)")
        if os.environ.get("GS_STALL_AT_STEP") is not None:
            # a rank that stops answering (the deadline's test): peers block in the barrier
            print(f"bench.py: rank {ctx.rank} stalls (GS_STALL_AT_STEP)", file=sys.stderr,
                  flush=True)
            time.sleep(1e6)
    ctx.barrier()
    sync()
    # the passes the timed window will run (a host-side query: engine.h plan_passes)
    timed_plan = sim.engine.plan_passes(args.steps) if hasattr(sim.engine, "plan_passes") else []
    _PROGRESS["phase"] = "timed region"
    t0 = time.perf_counter()
    sim.iterate(args.steps)
    sync()
    t1 = time.perf_counter()
    ctx.barrier()
    local = t1 - t0
    elapsed = ctx.allreduce(local, "max")
    stats = sim.global_stats()
    world_info = ctx.gather_object(sim.device_info())
    phases = None
    _PROGRESS["phase"] = "phase profile"
    if args.profile_passes > 0:
        # outside the timed region: the state it advances is reset by the golden check
        t_prof = time.perf_counter()
        phases = {"chosen": profile_phases(sim, ctx, args.profile_passes)}
        if ctx.world_size > 1 and backend == "hip":
            # the reference's Dims_create grid too, when the tuning chose another data path
            bal = dims_create(ctx.world_size)
            if list(dom.dims) != list(bal):
                rows = [r for r in (tuning or {}).get("table", []) if r["dims"] == bal
                        and r.get("ok")]
                phases["reference_grid"] = None
                if rows:
                    r = min(rows, key=lambda r: r["ms_per_step"])
                    # the same construction the tuning timed for this row; a failure is
                    # agreed by all ranks and recorded (the headline is already measured)
                    phases["reference_grid"] = profile_reference_grid(
                        settings, ctx, args, bal, r, args.profile_passes)
            from grayscott_amd.ops import native
            phases["peer_access"] = native.peer_access_matrix() if ctx.rank == 0 else None
        phases["profile_s"] = round(time.perf_counter() - t_prof, 2)
    if do_golden:
        _PROGRESS["phase"] = "golden check"
        t_chk = time.perf_counter()
        err = golden_check(sim, settings, dom, args.check_steps,
                           2024 if args.init == "random" else None)
        err = ctx.allreduce(err, "max")
        tol = 2e-5 if settings.dtype_name == "float32" else 1e-12
        check.update(golden_steps=args.check_steps, max_abs_err=err, golden_tol=tol,
                     golden_ok=bool(err < tol), golden_s=round(time.perf_counter() - t_chk, 2))
        if not err < tol:
            print(f"bench.py: golden check FAILED: max |gpu - golden| = {err:.3e} after "
                  f"{args.check_steps} steps (tolerance {tol:g})", file=sys.stderr, flush=True)
    cells = float(args.L) ** 3
    mlups = cells * args.steps / elapsed / 1e6
    if ctx.rank == 0:
        ref_grid = None
        if tuning:
            bal = dims_create(ctx.world_size)
            rows = [r for r in tuning["table"] if r["dims"] == bal and r.get("ok")]
            if rows:
                r = min(rows, key=lambda r: r["ms_per_step"])
                ref_grid = {"dims": bal, "fuse": r["fuse"], "overlapped": r.get("overlapped"),
                            "ms_per_step": r["ms_per_step"],
                            "mlups": round(cells / (r["ms_per_step"] * 1e-3) / 1e6, 1),
                            "steps_timed": r.get("steps")}
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
                "parallelism": parallelism_label(dom.dims, sim.transport, sim.overlapped,
                                                 sim.gated),
                "dims": dom.dims,
                "local_extent": dom.proc_sizes,
                "fuse_steps": sim.depth, "ghost_width": sim.H,
                "fused_kernel": {str(n): {"tile": c[0] or "default", "sched": c[1],
                                          "ms": round(float(c[2]), 4)}
                                 for n, c in sim.fused_choice().items()},
                # the timed window's passes (engine.h plan_passes; [] = greedy by fuse_steps)
                "pass_plan": timed_plan,
                # one outer-ghost refresh (ms): the planner's price of a depth-parity switch
                "bc_fill_ms": (round(sim.engine.fill_ms(), 4)
                               if hasattr(sim.engine, "fill_ms") else None),
                "transport": sim.transport,
                "overlap": sim.overlapped,
                "gated": sim.gated,
                "noise": args.noise,
                "backend": backend,
            },
            "world": {
                "ranks": ctx.world_size,
                "rccl_nranks": world_info[0].get("rccl_nranks"),
                "distinct_devices": len({w.get("pci") or w.get("device") for w in world_info}),
                "per_rank": world_info,
            },
            "tuning_s": round(tuning_s, 2),
            "wall_s": round(time.perf_counter() - T_START, 2),
            "data_path_tuning": tuning and tuning["table"],
            "link_probe": link,
            "reference_grid": ref_grid,
            "check": {"mean_u": stats["mean_u"], "mean_v": stats["mean_v"],
                      "finite": all(map(lambda x: x == x, stats.values())), **check},
        }
        if phases is not None:
            rec["phases"] = phases
        if ref_grid is not None and ctx.world_size == 8 and ref_grid["dims"] == [2, 2, 2]:
            rec["config3_2x2x2"] = ref_grid
        rec["status"] = "ok" if check.get("golden_ok", True) else "golden_check_failed"
        _emit_once(rec)
    _PROGRESS["phase"] = "teardown"
    sim.close()
    ctx.finalize()
    return 0 if check.get("golden_ok", True) else 1


if __name__ == "__main__":
    sys.exit(main())
