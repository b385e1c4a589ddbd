"""Multi-rank data-path selection: verify, then time, the candidate decompositions.

The reference has one data path (MPI_Dims_create grid + blocking host Sendrecv,
communication.jl:59-199).  Here several exist and the best one depends on the xGMI link rate
and RCCL's point-to-point latency, which differ between machines and cannot be measured on a
one-GPU box:

* z slabs ``1 x 1 x N``: halos are whole storage planes sent in place by RCCL and overlapped
  with the inner planes' update, but each rank moves ``2 * fuse`` full L x L planes per pass
  over just two links;
* the balanced ``MPI_Dims_create`` grid (2x2x2 on 8 GPUs): 4x less halo per link, spread over
  up to six links, but packed (pack / RCCL / unpack) and not overlapped;
* ``1 x 2 x N/2``: z slabs split once along y -- half the plane bytes per link, one tile ring;
* the fuse depth T (steps per exchange): the same bytes per step, fewer messages at larger T;
* the device transport: RCCL point-to-point, or the IPC peer-write transport (the pack kernel
  stores straight into the neighbours' landing buffers, device-side flags order the exchange;
  no RCCL kernel, no host handshake) -- its candidates carry ``transport = "ipc"``.

``tune_data_path`` first checks every candidate's exact data path against the golden model on
a small grid (``selfcheck``), then times a short run of each on the real problem, with every
rank agreeing on the winner (the time that counts is the slowest rank's).
"""
from __future__ import annotations

import contextlib
import copy
import os
import time
from typing import Dict, List, Optional, Sequence, Tuple

from .decomp import choose_dims, dims_create, init_domain


def selfcheck(ctx, backend: str, dims, fuse: int, transport: str, overlap: str, L: int = 64,
              steps: int = 15, precision: str = "Float32", skip_rccl: bool = False):
    """Run the exact data path (decomposition, transport, in-place halos, overlap, fuse depth,
    precision) on a small grid from the benchmarks' random init and compare with the
    numpy/torch golden model computed by every rank.  Returns ``(ok, max_abs_err,
    transport_used, error_text)``; ``ok`` and the error are agreed by all ranks.

    A rank that fails locally (set-up, a device wait that timed out, ...) still makes the same
    collectives as the others -- its error is reported as an infinite difference -- so the
    ranks' collective sequences never diverge.  ``skip_rccl``: the "auto" transport chain starts
    after RCCL (it failed to set up earlier on this node)."""
    import numpy as np

    from ..models.grayscott import GrayScott
    from ..ops import reference as ref
    from ..utils.config import Settings, parse_precision

    L = max(L, 8 * max(dims))
    err, used, text = float("inf"), None, None
    dtype = np.float32 if parse_precision(precision) == "float32" else np.float64
    try:
        s = Settings(L=L, precision=precision, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                     noise=0.1, backend="AMDGPU" if backend == "hip" else "CPU", seed=77,
                     transport=transport, overlap=overlap)
        dom = init_domain(L, ctx.world_size, ctx.rank, periodic=False, dims=dims)
        sim = GrayScott(s, dom, ctx, fuse=min(fuse, min(dom.proc_sizes)), skip_rccl=skip_rccl)
        try:
            sim.init_fields()
            sim.randomize_fields(seed=5)
            sim.iterate(steps)
            u, v = sim.get_fields()
            used = sim.transport
        finally:
            sim.close()
        ru, rv = ref.run(L, steps, noise_amp=0.1, seed=77, dtype=dtype, backend="torch",
                         init_seed=5)
        (ox, oy, oz), (nx, ny, nz) = dom.proc_offsets, dom.proc_sizes
        blk = (slice(oz, oz + nz), slice(oy, oy + ny), slice(ox, ox + nx))
        err = float(max(np.abs(u - ru[blk]).max(), np.abs(v - rv[blk]).max()))
        if not err == err:
            err = float("inf")
    except Exception as ex:  # reported, never raised past the collectives below
        text = str(ex)[:160]
    err = ctx.allreduce(err, "max")
    texts = [f"rank {r}: {t}" for r, t in enumerate(ctx.allgather_object(text)) if t]
    tol = 1e-4 if dtype == np.float32 else 1e-10
    return err < tol, err, used, ("; ".join(texts)[:240] or None)


def candidates(L: int, nprocs: int, backend: str) -> List[Tuple]:
    """(dims, fuse, overlap[, env[, transport]]) candidates worth timing for ``nprocs`` ranks on
    an L^3 grid (fuse 0 = auto; env: engine knobs set for that candidate; transport: a fixed
    halo transport instead of the run's own, with no fallback).  GS_TUNE_IPC=0 leaves out the
    IPC peer-write candidates."""
    out: List[Tuple] = []

    def add(d, f, ov="auto"):
        if (list(d), f, ov) not in out:
            out.append((list(d), f, ov))

    if nprocs == 1:
        return [([1, 1, 1], 0, "auto")]
    z = choose_dims(L, nprocs, "z", backend)
    bal = dims_create(nprocs)
    # the reference's Dims_create grid first: it is always timed (bench.py reports it as
    # ``reference_grid``), then the z slabs (overlapped and not: the overlap's split launches
    # cost more than they hide unless the exchange is slow), then the variants.  Fuse depth 2
    # never won a z-slab row at L=512 (profiles/r3_rehearsal_pre.txt, round-2 tables); on the
    # balanced grid it halves the overlapped pass's face-slab shell (11 vs 28 us per pass for a
    # 256^3 rank, profiles/r3_overlap_split.txt), so it is timed there.
    add(bal, 0)
    if backend == "hip" and L // nprocs >= 8:
        add(z, 0)
        add(z, 0, "off")
    if backend == "hip":
        add(bal, 0, "off")
        add(bal, 2)
        # z slabs split once along y: half the z-plane bytes per link of the plain slabs, full
        # 64-lane x tiles, and only one face slab (y) outside the overlap
        if nprocs >= 4 and nprocs % 2 == 0 and L // (nprocs // 2) >= 8:
            add([1, 2, nprocs // 2], 0)
            add([1, 2, nprocs // 2], 0, "off")
        # the IPC peer-write transport on the two main grids, overlapped and not
        if os.environ.get("GS_TUNE_IPC", "1") != "0":
            if L // nprocs >= 8:
                out.append((list(z), 0, "auto", {}, "ipc"))
                out.append((list(z), 0, "off", {}, "ipc"))
            out.append((list(bal), 0, "auto", {}, "ipc"))
            out.append((list(bal), 0, "off", {}, "ipc"))
            out.append((list(bal), 2, "auto", {}, "ipc"))
    return out


# A candidate the model says loses by more than this factor is not timed (link-probe pruning)
MODEL_PRUNE = 1.20
# What an overlapped pass costs on top of max(update, exchange), as a share of the update, per
# halo layout and transport (measured on one GPU with the exchange in flight):
#   IPC: gated passes (the exchange inside the pass's launch) -- z slab 1.05-1.07x, 2x2x2 rank
#        1.11-1.15x the full pass (profiles/r5_gated.txt);
#   RCCL: stream-overlapped passes (inner box, then the face-slab shell) -- 2x2x2 rank 1.34x
#        (README round-4 item 3, profiles/r4_shell.txt); z slabs only split off their two faces
#        (profiles/r3_overlap_split.txt: 11-28 us shells on ~560 us passes)
OVERLAP_COST = {("zslab", "ipc"): 0.07, ("zslab", "rccl"): 0.10,
                ("packed", "ipc"): 0.15, ("packed", "rccl"): 0.34}


def overlap_cost(dims, transport: str) -> float:
    zslab = int(dims[0]) == 1 and int(dims[1]) == 1
    return OVERLAP_COST[("zslab" if zslab else "packed", "ipc" if transport == "ipc" else "rccl")]


def pass_messages(dom, H: int) -> List[int]:
    """Cells this rank sends to each neighbour per pass of depth ``H``: a face H x n x n, an edge
    H x H x n, a corner H^3 -- and on z slabs (process grid 1 x 1 x N) whole storage planes,
    x / y ghosts included (the in-place plane halos, engine.h halo plan)."""
    nx, ny, nz = dom.proc_sizes
    zslab = dom.dims[0] == 1 and dom.dims[1] == 1
    out = []
    for i, r in enumerate(dom.nbr27):
        if i == 13 or r < 0 or r == dom.rank:
            continue
        dx, dy, dz = i // 9 - 1, (i // 3) % 3 - 1, i % 3 - 1
        if zslab:
            out.append(H * (nx + 2 * H) * (ny + 2 * H))
            continue
        ex = H if dx else nx
        ey = H if dy else ny
        ez = H if dz else nz
        out.append(ex * ey * ez)
    return out


def model_step_ms(L: int, nprocs: int, dims, fuse: int, overlap: str, transport: str,
                  link: Optional[Dict], comp_step_ms: float, pair_bytes: int = 8) -> Optional[float]:
    """Modelled ms per step of a candidate: every rank's pass is its update (``fuse`` steps of
    ``comp_step_ms``, the same local volume on every candidate) plus its exchange -- the slowest
    of its neighbour messages over the slowest probed link of ``transport`` (xGMI links are
    point to point: the messages to different neighbours move at once) -- in sequence, or
    overlapped (max of the two plus overlap_cost of the update) unless ``overlap`` is "off".
    The slowest rank sets the pace.  None if the link probe has no rates for ``transport``."""
    from .linkprobe import transfer_us
    H = max(1, int(fuse))
    comp = comp_step_ms * H
    oc = overlap_cost(dims, transport)
    worst = 0.0
    for r in range(nprocs):
        dom = init_domain(L, nprocs, r, periodic=False, dims=dims)
        xs = [transfer_us(link, transport, c * pair_bytes) for c in pass_messages(dom, H)]
        if any(x is None for x in xs):
            return None
        xch = max(xs, default=0.0) * 1e-3
        t = comp + xch if overlap == "off" else max(comp, xch) + oc * comp
        worst = max(worst, t)
    return worst / H


def prune_by_model(pred: Dict[int, float], protected: Sequence[int],
                   factor: float = MODEL_PRUNE) -> Dict[int, float]:
    """The candidates (index -> modelled ms per step) the model rules out: those slower than
    ``factor`` x the best modelled candidate, except the ``protected`` ones (the reference's
    Dims_create grid is always timed).  Returns index -> modelled slowdown."""
    if not pred:
        return {}
    best = min(pred.values())
    return {i: round(t / best, 3) for i, t in pred.items()
            if i not in protected and best > 0 and t > factor * best}


def time_data_path(settings, ctx, L: int, dims, fuse: int, steps: int = 30, warmup: int = 6,
                   seed: int = 2024, skip_rccl: bool = False, info: Optional[Dict] = None):
    """(seconds for ``steps`` steps of the real problem on this data path (max over ranks),
    whether its passes overlap the halo exchange).  ``info`` (optional) receives
    ``comp_ms_per_step``: the update alone, the fused pass time the engine's autotuner measured
    on this rank's block at the pass depth, per step (max over ranks; 0 if untimed)."""
    import torch

    from ..models.grayscott import GrayScott

    s = copy.copy(settings)
    s.fuse_steps = int(fuse)
    dom = init_domain(L, ctx.world_size, ctx.rank, periodic=False, dims=dims)
    sim = GrayScott(s, dom, ctx, skip_rccl=skip_rccl)
    try:
        sim.init_fields()
        sim.randomize_fields(seed=seed)

        def sync():
            sim.synchronize()
            if sim.backend == "hip":
                torch.cuda.synchronize()

        sim.iterate(warmup)
        sync()
        ctx.barrier()
        t0 = time.perf_counter()
        sim.iterate(steps)
        sync()
        el = time.perf_counter() - t0
        ovd = "gated" if sim.gated else bool(sim.overlapped)  # gated: the exchange in-kernel
        c = sim.fused_choice().get(int(sim.depth)) if sim.backend == "hip" else None
        comp = float(c[2]) / max(1, int(sim.depth)) if c and c[2] else 0.0
    finally:
        sim.close()
    comp = ctx.allreduce(comp, "max")
    if info is not None:
        info["comp_ms_per_step"] = comp
    return ctx.allreduce(el, "max"), ovd


def tune_data_path(settings, ctx, L: int, backend: str,
                   cands: Optional[Sequence[Tuple]] = None,
                   steps: int = 120, warmup: int = 12, log=None,
                   budget_s: Optional[float] = None, on_row=None,
                   link: Optional[Dict] = None) -> Dict:
    """Self-check and time every candidate ``(dims, fuse[, overlap[, env]])``; returns
    ``{"dims", "fuse", "transport", "overlap", "inplace_halos", "env", "table"}`` for the fastest
    correct one (identical on every rank; ``env`` must be set for the run that uses it).

    ``budget_s`` bounds the whole tuning phase: once it is spent (rank 0's clock, agreed by all
    ranks) the remaining candidates are skipped (``"skipped": "budget"`` in the table), but at
    least two are always tried.  Once one candidate's transport passed its check, later
    candidates do not retry the fallback transports: a failure there is the path's own.

    Fail fast per transport: once a pinned transport (IPC) fails a candidate's check with a
    transport-level error on some rank -- a peer wait that timed out, a mapping or set-up
    error -- every later candidate pinned to it is skipped (``"skipped": "ipc failed:
    <reason>"``), so a node whose cross-device IPC misbehaves pays its timeout once, not once
    per IPC row.  A numerical mismatch is the candidate's own (its grid, overlap mode or tile):
    later rows on the same transport are still tried.  Likewise, once RCCL failed to set up,
    later candidates' fallback chains start after it (``skip_rccl``).  ``on_row(row)`` is
    called with every finished table row (bench.py streams them for a failure report).

    Link-probe pruning (``link``: parallel/linkprobe.py probe_links, the same dict on every
    rank):
      * once a row is timed, the fused pass time its engine's autotuner measured on the rank's
        block fixes the update cost per step (``model_comp_ms_per_step``), and every later
        candidate gets a modelled time (``model_ms_per_step``, model_step_ms).  Those more than
        MODEL_PRUNE x the best modelled candidate are recorded as ``"skipped": "model"`` instead
        of being checked and timed; the reference's Dims_create grid rows never are (BASELINE
        config 3 is always measured);
      * where the probe found RCCL unusable but IPC working, the IPC rows are timed first, and
        once one passed, the rows without a pinned transport (whose "auto" chain would fall back
        to the host-staged transport) are skipped (``"skipped": "rccl unavailable"``).
    GS_TUNE_MODEL=0 turns the pruning off (the predictions are still recorded)."""
    from ..models.grayscott import default_fuse

    cands = list(cands) if cands is not None else candidates(L, ctx.world_size, backend)
    table = []
    best = None
    bal = dims_create(ctx.world_size)
    pair_bytes = 8 if settings.dtype_name == "float32" else 16
    use_model = link is not None and os.environ.get("GS_TUNE_MODEL", "1") != "0"
    comp_step = None  # ms per step of the update alone (from the first timed row)
    # (only where the run's own transport would try RCCL first: an explicit host / torch / IPC
    # transport is what the user asked to time)
    no_rccl = bool(use_model and link.get("rccl_failed") and link.get("ipc") == "ok" and
                   str(settings.transport).lower() in ("auto", "rccl"))
    if no_rccl:
        # the IPC rows first, in their own order (the rows after them that fall back to the host
        # transport are skipped once one IPC row passed)
        cands = ([c for c in cands if len(c) > 4 and c[4] == "ipc"] +
                 [c for c in cands if not (len(c) > 4 and c[4] == "ipc")])

    def resolved(cand):
        dom = init_domain(L, ctx.world_size, ctx.rank, periodic=False, dims=cand[0])
        f = cand[1] if cand[1] > 0 else default_fuse(backend, dom, settings.dtype_name)
        f = max(1, min(f, min(dom.proc_sizes)))
        ov = cand[2] if len(cand) > 2 else settings.overlap
        tr = cand[4] if len(cand) > 4 and cand[4] else "rccl"
        return f, ov, tr

    def predict(cand):
        if comp_step is None or link is None:
            return None
        f, ov, tr = resolved(cand)
        return model_step_ms(L, ctx.world_size, cand[0], f, ov, tr, link, comp_step, pair_bytes)

    pruned: Dict[int, float] = {}
    t_start = time.perf_counter()
    proven = None  # transport that passed a check on this node
    failed: Dict[str, str] = {}  # pinned transport -> why it failed on this node

    def finish(row):
        table.append(row)
        if on_row is not None:
            on_row(row)

    for ci, cand in enumerate(cands):
        over = budget_s is not None and time.perf_counter() - t_start > budget_s
        if ci >= 2 and ctx.allreduce(1.0 if over else 0.0, "max") > 0:
            finish({"dims": list(cand[0]), "fuse": cand[1],
                    "overlap_req": cand[2] if len(cand) > 2 else settings.overlap,
                    "skipped": "budget"})
            continue
        if no_rccl and not (len(cand) > 4 and cand[4]) and any(
                r.get("ok") and r.get("transport") == "ipc" for r in table):
            finish({"dims": list(cand[0]), "fuse": resolved(cand)[0],
                    "overlap_req": cand[2] if len(cand) > 2 else settings.overlap,
                    "skipped": "rccl unavailable (link probe): host fallback not timed"})
            continue
        if ci in pruned:
            finish({"dims": list(cand[0]), "fuse": resolved(cand)[0],
                    "overlap_req": cand[2] if len(cand) > 2 else settings.overlap,
                    **({"transport_req": cand[4]} if len(cand) > 4 and cand[4] else {}),
                    "skipped": "model", "model_ms_per_step": round(predict(cand), 4),
                    "model_slowdown": pruned[ci]})
            continue
        dims, fuse = cand[0], cand[1]
        ov0 = cand[2] if len(cand) > 2 else settings.overlap
        env0 = dict(cand[3]) if len(cand) > 3 else {}
        tr0 = cand[4] if len(cand) > 4 else None
        dom = init_domain(L, ctx.world_size, ctx.rank, periodic=False, dims=dims)
        f = fuse if fuse > 0 else default_fuse(backend, dom, settings.dtype_name)
        f = max(1, min(f, min(dom.proc_sizes)))
        if any(r["dims"] == list(dims) and r["fuse"] == f and r["overlap_req"] == ov0
               and r.get("env", {}) == env0 and r.get("transport_req") == tr0 for r in table):
            continue  # "auto" resolved to a depth already in the list
        row = {"dims": list(dims), "fuse": f, "overlap_req": ov0}
        if env0:
            row["env"] = env0
        if tr0:
            row["transport_req"] = tr0
        if tr0 and tr0 in failed:
            # (every rank holds the same `failed`: it is built from agreed results only)
            row["skipped"] = f"{tr0} failed: {failed[tr0]}"
            row["ok"] = False
            finish(row)
            continue
        chosen = None
        attempts = [(settings.transport, ov0, {}),
                    (settings.transport, "off", {"GS_INPLACE_HALO": "0"}),
                    ("torch", "off", {"GS_INPLACE_HALO": "0"})]
        if backend == "hip":
            attempts.append(("host", "off", {"GS_INPLACE_HALO": "0"}))
        if proven is not None:
            attempts = [(proven, ov0, {})]
        if tr0:
            # a fixed transport: no fallback chain; a peer that never signals ends its device
            # waits after 20 s instead of GS_COMM_TIMEOUT
            attempts = [(tr0, ov0, {"GS_COMM_TIMEOUT": "20"})]
        # the fallback chain of "auto" starts after RCCL once its set-up failed on this node
        skip_rccl = "rccl" in failed
        for tr, ov, extra in attempts:
            env = {**env0, **extra}
            with _env(env):
                # selfcheck never raises and makes the same collectives on every rank
                ok, err, used, text = selfcheck(ctx, backend, dims, f, tr, ov,
                                                precision=settings.precision,
                                                skip_rccl=skip_rccl)
            if not ok:
                # reported in the bench JSON (data_path_tuning): why a transport failed
                row.setdefault("check_errors", []).append(
                    f"{tr}: {text}" if text else f"{tr}: max |err| {err:.3g} vs golden")
            ok = ctx.allreduce(1.0 if ok else 0.0, "min") > 0
            # agreed failure reasons (every rank the same): rank 0's text, or the mismatch
            why = ctx.broadcast_object((text or f"max |err| {err:.3g} vs golden")[:120], src=0)
            # a transport-level failure: some rank raised (set-up, mapping, a wait that timed
            # out); a pure mismatch raised nowhere (selfcheck's error text stays None)
            raised = ctx.allreduce(1.0 if text else 0.0, "max") > 0
            if not ok and tr0 and raised:
                failed[tr0] = why
            if not ok and "rccl" in why.lower() and ("init" in why.lower() or
                                                     "unique" in why.lower()):
                failed["rccl"] = why
            if ok:
                chosen = (used, ov, {**env0, **(extra if not tr0 else {})})
                if not extra and not tr0:
                    proven = used
                break
        if chosen is None:
            row.update(ok=False)
            finish(row)
            continue
        s = copy.copy(settings)
        s.transport, s.overlap = chosen[0], chosen[1]
        tinfo: Dict = {}
        with _env(chosen[2]):
            try:
                el, ovd = time_data_path(s, ctx, L, dims, f, steps=steps, warmup=warmup,
                                         skip_rccl=skip_rccl, info=tinfo)
                ran = 1.0
            except Exception as ex:  # e.g. out of memory at the real size: skip this path
                el, ovd, ran = float("inf"), False, 0.0
                row["error"] = str(ex)[:200]
        if ctx.allreduce(ran, "min") <= 0:
            row.update(ok=False)
            finish(row)
            continue
        row.update(ok=True, transport=chosen[0], overlap=chosen[1], overlapped=ovd,
                   inplace_halos=chosen[2].get("GS_INPLACE_HALO") != "0",
                   ms_per_step=round(1e3 * el / steps, 4), steps=steps)
        if link is not None and comp_step is None and tinfo.get("comp_ms_per_step", 0) > 0:
            # the update's own cost per step: the tuned fused pass on this row's blocks (every
            # candidate updates the same L^3 / N cells per rank)
            ms = 1e3 * el / steps
            comp_step = float(tinfo["comp_ms_per_step"])
            row["model_comp_ms_per_step"] = round(comp_step, 4)
            preds = {}
            for cj, cc in enumerate(cands):
                if cj > ci:
                    pj = predict(cc)
                    if pj is not None:
                        preds[cj] = pj
            preds[ci] = predict(cand) or ms
            protected = [cj for cj, cc in enumerate(cands) if list(cc[0]) == list(bal)]
            if use_model:
                pruned = prune_by_model(preds, protected)
        pj = predict(cand)
        if pj is not None:
            row["model_ms_per_step"] = round(pj, 4)
        finish(row)
        if log is not None and ctx.rank == 0:
            log(f"data path {row}")
        if best is None or el < best[0]:
            best = (el, list(dims), f, chosen)
    if best is None:
        raise RuntimeError(f"no multi-rank data path passed its self-check: {table}")
    env = best[3][2]
    if log is not None and ctx.rank == 0:
        log(f"data-path tuning took {time.perf_counter() - t_start:.1f} s")
    return {"dims": best[1], "fuse": best[2], "transport": best[3][0], "overlap": best[3][1],
            "inplace_halos": env.get("GS_INPLACE_HALO") != "0", "env": env, "table": table}


@contextlib.contextmanager
def _env(overrides: Dict[str, str]):
    """Environment knobs read at engine creation (GS_INPLACE_HALO, GS_COMM_TIMEOUT, ...)
    set for one candidate and restored afterwards."""
    old = {k: os.environ.get(k) for k in overrides}
    os.environ.update(overrides)
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
