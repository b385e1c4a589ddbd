"""Link probe: every pair of ranks measures its own GPU-to-GPU path before the data-path tuner
times a candidate (csrc/hip/probe.hpp does the device side).

The reference exchanges halos one way and never measures it (``communication.jl:138-199``,
blocking ``MPI.Sendrecv!``).  Here the tuner (``parallel/autotune.py``) picks between z slabs and
the reference's ``Dims_create`` grid, RCCL and IPC peer stores, overlapped or not -- and the
right pick depends on what one xGMI link delivers at the message sizes those candidates send:

* z slabs send whole planes, 6.3 MB per neighbour per T=3 pass for a 512^2 fp32 plane pair;
* the 2x2x2 grid sends 1.5 MB faces (and small edges / corners) over up to seven links.

So each pair measures, both directions at once (as in an exchange), the time of a put of each
probe size through IPC peer stores and through an RCCL send / receive pair.  The pairs are
scheduled round-robin (circle method: ``world - 1`` rounds of disjoint pairs), so no link is
shared within a round.  The result -- identical on every rank -- is reported as ``link_probe``
in the bench JSON and feeds ``autotune.model_step_ms``, which keeps the tuner from timing
candidates its model says lose by more than 20 %.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence, Tuple

# probe sizes (bytes): a small put (launch + link latency), one 256^2 fp32 pair plane (a
# 2x2x2 face at T=1), a 2x2x2 face at T=3 (256^2 x 3 x 8 B) and a z-slab message at T=3
# (512^2 x 3 x 8 B)
PROBE_SIZES = (4096, 256 * 256 * 8, 256 * 256 * 3 * 8, 512 * 512 * 3 * 8)


def round_robin(n: int) -> List[List[Tuple[int, int]]]:
    """Rounds of disjoint pairs covering every pair of ``n`` ranks once (circle method; odd
    ``n``: one rank sits out each round)."""
    if n < 2:
        return []
    m = n if n % 2 == 0 else n + 1
    ring = list(range(m))
    rounds = []
    for _ in range(m - 1):
        pairs = []
        for i in range(m // 2):
            a, b = ring[i], ring[m - 1 - i]
            if a < n and b < n:
                pairs.append((min(a, b), max(a, b)))
        rounds.append(sorted(pairs))
        ring = [ring[0], ring[-1]] + ring[1:-1]
    return rounds


def _partner(pairs: Sequence[Tuple[int, int]], rank: int) -> Optional[int]:
    for a, b in pairs:
        if a == rank:
            return b
        if b == rank:
            return a
    return None


def probe_links(ctx, sizes: Sequence[int] = PROBE_SIZES, reps: int = 5, rccl: bool = True,
                log=None) -> Optional[Dict]:
    """Measure every pair's IPC peer-store and RCCL send / receive times (HIP ranks only; None
    with one rank).  Every rank takes part in the same collectives whatever fails locally, and
    every rank returns the same dict:
      ``pairs``: per pair {ranks, pci, ipc_us, ipc_GBps, rccl_us, rccl_GBps} (per size);
      ``summary``: per transport and size the slowest pair's GB/s (``*_GBps_min``) and the
      median, and the slowest 4 KB put (``*_small_us_max``);
      ``rccl``: "ok" or why the communicator could not be set up (``rccl_failed`` True then);
      ``probe_s``: the probe's wall time."""
    if ctx.world_size < 2:
        return None
    from ..ops import native

    t0 = time.perf_counter()
    sizes = [int(s) for s in sizes]
    rounds = round_robin(ctx.world_size)
    mine: Dict[str, Dict] = {"ipc": {}, "rccl": {}}
    err: Dict[str, Optional[str]] = {"ipc": None, "rccl": None}
    probe = None
    try:
        probe = native.LinkProbe(max(sizes))
        exp = probe.export()
    except Exception as ex:  # reported; the collectives below still run
        exp = b""
        err["ipc"] = f"rank {ctx.rank}: {ex}"[:200]
    exports = ctx.allgather_object(exp)
    pcis = ctx.allgather_object(native.device_pci_bus_id())
    ipc_ok = ctx.allreduce(0.0 if err["ipc"] else 1.0, "min") > 0
    if ipc_ok:
        for pairs in rounds:
            peer = _partner(pairs, ctx.rank)
            for s in sizes:
                ctx.barrier()  # both directions of every pair at once
                if peer is None or err["ipc"]:
                    continue
                try:
                    mine["ipc"][(peer, s)] = probe.ipc_us(exports[peer], s, reps)
                except Exception as ex:
                    err["ipc"] = f"rank {ctx.rank} -> {peer}: {ex}"[:200]
    rccl_state = "not probed"
    # every rank takes the same branch (a rank whose probe buffers failed must not skip the
    # collectives its peers make below)
    have = ctx.allreduce(1.0 if probe is not None else 0.0, "min") > 0
    if rccl and have:
        uid = None
        if ctx.rank == 0:
            try:
                uid = native.rccl_unique_id()
            except Exception as ex:  # broadcast as None: every rank reports the failure
                err["rccl"] = f"rank 0: {ex}"[:200]
        uid = ctx.broadcast_object(uid, src=0)
        try:
            if uid is None:
                raise RuntimeError("no RCCL unique id (rank 0 could not create one)")
            probe.rccl_init(uid, ctx.world_size, ctx.rank)
        except Exception as ex:
            err["rccl"] = err["rccl"] or f"rank {ctx.rank}: {ex}"[:200]
        rccl_ok = ctx.allreduce(0.0 if err["rccl"] else 1.0, "min") > 0
        if rccl_ok:
            for pairs in rounds:
                peer = _partner(pairs, ctx.rank)
                for s in sizes:
                    ctx.barrier()
                    if peer is None or err["rccl"]:
                        continue
                    try:
                        mine["rccl"][(peer, s)] = probe.rccl_us(peer, s, reps)
                    except Exception as ex:
                        err["rccl"] = f"rank {ctx.rank} <-> {peer}: {ex}"[:200]
        texts = [e for e in ctx.allgather_object(err["rccl"]) if e]
        rccl_state = "ok" if not texts else texts[0]
    if probe is not None:
        probe.close()
    allm = ctx.allgather_object({k: {f"{p}:{s}": t for (p, s), t in v.items()}
                                 for k, v in mine.items()})
    ipc_texts = [e for e in ctx.allgather_object(err["ipc"]) if e]
    out = summarize(allm, pcis, sizes, rounds)
    out.update(rccl=rccl_state, rccl_failed=rccl_state not in ("ok", "not probed"),
               ipc="ok" if not ipc_texts else ipc_texts[0],
               probe_s=round(ctx.allreduce(time.perf_counter() - t0, "max"), 3))
    if log is not None and ctx.rank == 0:
        log(f"link probe: {out['summary']} ({out['probe_s']} s)")
    return out


def summarize(allm: Sequence[Dict], pcis: Sequence[str], sizes: Sequence[int],
              rounds: Sequence[Sequence[Tuple[int, int]]]) -> Dict:
    """Pair table and summary from every rank's times ``allm[rank][transport]["peer:size"]``
    (microseconds; a pair's time at a size is the slower of its two directions)."""
    pairs_out = []
    per = {"ipc": {s: [] for s in sizes}, "rccl": {s: [] for s in sizes}}
    for pairs in rounds:
        for a, b in pairs:
            row = {"ranks": [a, b], "pci": [pcis[a], pcis[b]]}
            for tr in ("ipc", "rccl"):
                us, gbs = {}, {}
                for s in sizes:
                    ta = allm[a].get(tr, {}).get(f"{b}:{s}")
                    tb = allm[b].get(tr, {}).get(f"{a}:{s}")
                    if ta is None or tb is None:
                        continue
                    t = max(ta, tb)
                    us[str(s)] = round(t, 2)
                    gbs[str(s)] = round(s / (t * 1e3), 2) if t > 0 else None
                    per[tr][s].append(t)
                if us:
                    row[f"{tr}_us"], row[f"{tr}_GBps"] = us, gbs
            pairs_out.append(row)
    summary = {}
    for tr in ("ipc", "rccl"):
        if not any(per[tr][s] for s in sizes):
            continue
        worst = {str(s): round(max(per[tr][s]), 2) for s in sizes if per[tr][s]}
        med = {str(s): round(sorted(per[tr][s])[len(per[tr][s]) // 2], 2)
               for s in sizes if per[tr][s]}
        summary[f"{tr}_us_max"] = worst
        summary[f"{tr}_GBps_min"] = {k: round(int(k) / (v * 1e3), 2) for k, v in worst.items()
                                     if v > 0}
        summary[f"{tr}_GBps_median"] = {k: round(int(k) / (v * 1e3), 2) for k, v in med.items()
                                        if v > 0}
        small = min(sizes)
        if per[tr][small]:
            summary[f"{tr}_small_us_max"] = round(max(per[tr][small]), 2)
    return {"sizes": list(sizes), "pairs": pairs_out, "summary": summary}


def transfer_us(link: Optional[Dict], transport: str, nbytes: float) -> Optional[float]:
    """Modelled time (us) of one message of ``nbytes`` over the slowest probed pair of
    ``transport`` ("ipc" / "rccl"): piecewise linear in the probed (size, time) points, the
    largest size's rate beyond it, the smallest size's time below it.  None if not probed."""
    if not link:
        return None
    worst = link.get("summary", {}).get(f"{transport}_us_max")
    if not worst:
        return None
    pts = sorted((int(k), float(v)) for k, v in worst.items())
    if nbytes <= 0:
        return 0.0
    if nbytes <= pts[0][0]:
        return pts[0][1]
    for (s0, t0), (s1, t1) in zip(pts, pts[1:]):
        if nbytes <= s1:
            return t0 + (t1 - t0) * (nbytes - s0) / (s1 - s0)
    s, t = pts[-1]
    return t * nbytes / s
