"""The Gray-Scott model: fields + native engine for one rank.

Reference façade being replaced:
  * ``init_fields(settings, mcd, T)``      -- public.jl:18-25 and the per-backend inits
                                              (Simulation_CPU.jl:14-65, ext/*Ext.jl populate!)
  * ``iterate!(fields, settings, mcd)``    -- public.jl:45-71 (exchange! -> calculate! -> swap)
  * ``get_fields(backend, fields)``        -- Simulation_CPU.jl:125-133, ext/CUDAExt.jl:199-209
  * ``Fields{T,N,A}``                      -- Structs.jl:82-93

Fields live in one interleaved (u, v) buffer pair per rank, allocated as torch tensors (device
memory on MI355X, host memory for the CPU backend) and updated in place by the native engine.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np
import torch

from ..ops import native
from ..parallel.decomp import CartDomain
from ..parallel.dist import DistContext
from ..parallel.halo import TorchTransport
from ..utils.config import Settings, load_backend_and_lang, parse_precision

_TORCH_DTYPES = {"float32": torch.float32, "float64": torch.float64}
# set (identically on every rank: the chain's outcome is agreed) once RCCL failed its set-up or
# trial exchange in this process's "auto" transport chain: later engines skip it instead of
# paying its GS_COMM_TIMEOUT again (the data-path tuner builds a dozen engines)
_RCCL_FAILED = [False]
_NP_DTYPES = {"float32": np.float32, "float64": np.float64}


def default_fuse(backend: str, domain: CartDomain, dtype: str = "float32") -> int:
    """Steps fused per halo exchange when ``fuse_steps = 0`` (auto)."""
    if backend != "hip":
        return 1
    # The temporally blocked kernel cuts HBM traffic per step by T; a deeper halo also cuts
    # the RCCL round trips.  Measured on MI355X with the round-2 kernel
    # (profiles/r2_fuse_small.txt; round 1: profiles/r1_tune_fuse_depth.txt): T=3 wins from
    # 192^2 x-y planes up (L=192: 407-411k vs 370-403k MLUPS, L=256: 495-505k vs 459-468k);
    # T=2 on smaller planes (L=128: 224-227k vs 191-192k, L=64: 54k vs 42k), where the
    # 2T-cell tile halo costs more than the saved traffic.  fp64 follows the same rule since
    # round 3 (T=2 is HBM-bound there: L=512 344k vs 311k MLUPS, L=1024 332k vs 276k at T=3,
    # profiles/r3_f64_depth.txt; round 1 measured the opposite, profiles/r1_tune_f64.txt).
    nx, ny, nz = domain.proc_sizes
    if not any(r >= 0 and r != domain.rank for i, r in enumerate(domain.nbr27) if i != 13):
        # no halo exchange to amortise: H = 3 ghost layers (fp32: 4, the LDS-ring kernel's T = 4
        # entry), prepare() times every depth and each iterate(n) runs the partition of n into
        # passes with the lowest summed measured time (engine.h plan_passes) -- the block
        # kernel (csrc/hip/block.hpp) moved the small-grid crossover
        return max(1, min(4 if dtype == "float32" else 3, nx, ny, nz))
    t = 2 if min(nx, ny) < 160 else 3
    return max(1, min(t, nx, ny, nz))



def critical_path(ph: dict, xch: float, per_pass: dict, chained: bool) -> float:
    """Critical path of one pass (us) from its median phase times ``ph``, the exchange span
    ``xch`` and the share of passes each phase ran in (``per_pass``):
      * chained overlapped passes (engine.h advance_chained): inner_p waits for shell_{p-1},
        shell_p for exchange_p and inner_{p-1}, so the steady-state period is
        max(inner, exchange + shell);
      * one overlapped pass at a time: max(inner, exchange) + shell;
      * otherwise the phases run in sequence: exchange + fused + step.
    A phase that runs in some passes only (the boundary refill after a depth change) counts
    with its share of the passes."""
    bc = ph.get("bc", 0.0) * min(1.0, per_pass.get("bc", 0.0))
    if "inner" in ph or "shell" in ph:
        inner, shell = ph.get("inner", 0.0), ph.get("shell", 0.0)
        if chained:
            return max(inner, xch + shell) + bc
        return max(inner, xch) + shell + bc
    return xch + ph.get("fused", 0.0) + ph.get("step", 0.0) + bc


def _agree_gated_depths(engine, ctx, fuse: int) -> dict:
    """Gated passes (csrc/hip/gate.hpp) per depth on every rank or on none.  Every depth 2..fuse
    can run gated -- prepare() tunes each, and a planned or remainder pass of any depth takes the
    gated path where gated(k) holds -- and gated_supported(k) depends on per-rank state (the
    sub-domain's planes, the per-depth occupancy, shared landing slots).  One allreduce of the
    per-depth mask (min over ranks); the depths some rank cannot run gated are switched off on
    every rank (engine.h set_gated_depth).  Returns {depth: agreed}."""
    ks = list(range(2, max(2, int(fuse)) + 1))
    mine = [1.0 if engine.gated(k) else 0.0 for k in ks]
    agreed = ctx.allreduce_array(mine, "min")
    out = {}
    for k, a in zip(ks, agreed):
        on = a > 0
        if not on:
            engine.set_gated_depth(k, False)
        out[k] = on
    return out


class GrayScott:
    """One rank's Gray-Scott state and stepping engine."""

    def __init__(self, settings: Settings, domain: CartDomain, ctx: Optional[DistContext] = None,
                 fuse: Optional[int] = None, transport: Optional[str] = None,
                 use_fused: bool = True, loopback: bool = False, skip_rccl: bool = False):
        self.settings = settings
        self.domain = domain
        self.ctx = ctx or DistContext()
        self.backend, self.kernel_language = load_backend_and_lang(settings)
        self.dtype = parse_precision(settings.precision)
        if self.backend == "hip":
            if not torch.cuda.is_available():
                raise RuntimeError("backend requests the MI355X HIP path but no GPU is visible")
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")
        auto_depth = (fuse is None or fuse <= 0) and settings.fuse_steps <= 0
        if fuse is None or fuse <= 0:
            fuse = (settings.fuse_steps if settings.fuse_steps > 0
                    else default_fuse(self.backend, domain, parse_precision(settings.precision)))
        fuse = int(max(1, min(fuse, min(domain.proc_sizes))))
        self.fuse = fuse
        self.H = fuse
        nx, ny, nz = domain.proc_sizes
        ox, oy, oz = domain.proc_offsets
        Lx, Ly, Lz = domain.L
        self.geom = native.make_geom(nx, ny, nz, self.H, ox, oy, oz, Lx, Ly, Lz, domain.periodic)
        n = native.total_elems(self.geom)
        tdt = _TORCH_DTYPES[self.dtype]
        # zeroed once so the row padding never holds garbage (it is never read for valid cells)
        self.buffers = [torch.zeros(2 * n, dtype=tdt, device=self.device) for _ in range(2)]
        scells, rcells = native.plan_sizes(self.geom, domain.nbr27, self.H > 1)
        self.sendbuf = torch.empty(max(2 * scells, 2), dtype=tdt, device=self.device)
        self.recvbuf = torch.empty(max(2 * rcells, 2), dtype=tdt, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream if self.backend == "hip" else 0
        p = native.Params()
        p.F, p.k, p.dt = settings.F, settings.k, settings.dt
        p.Du, p.Dv, p.noise = settings.Du, settings.Dv, settings.noise
        p.seed = int(settings.seed) & 0xFFFFFFFFFFFFFFFF
        self.params = p
        self.engine = native.Engine(self.backend, self.dtype, self.geom, p, domain.nbr27,
                                    domain.rank, fuse, use_fused, self.buffers[0].data_ptr(),
                                    self.buffers[1].data_ptr(), self.sendbuf.data_ptr(),
                                    self.recvbuf.data_ptr(), stream)
        # a depth left to the engine: prepare() may run fewer steps per pass when they are
        # cheaper per step (single rank; an explicit fuse is kept as given)
        self.engine.set_auto_depth(auto_depth)
        ov = str(getattr(settings, "overlap", "auto")).lower()
        if ov not in ("auto", "on", "off", "true", "false", "1", "0"):
            raise ValueError(f"overlap must be auto | on | off, not {ov!r}")
        self.engine.set_overlap(-1 if ov == "auto" else (1 if ov in ("on", "true", "1") else 0))
        self.transport = "none"
        # the data-path tuner's candidates after RCCL failed to set up on this node: the "auto"
        # transport chain starts after it (parallel/autotune.py)
        self._skip_rccl = bool(skip_rccl)
        if loopback:
            # single-GPU test mode: the periodic wraps onto this rank go through RCCL
            # send/recv-to-self, exercising the multi-rank data path (engine.h set_loopback)
            if not domain.has_neighbors:
                raise ValueError("loopback needs a domain with (periodic) neighbours")
            self.engine.set_loopback(True)
            self._setup_transport(transport or "rccl")
        elif domain.has_neighbors and any(r != domain.rank for i, r in enumerate(domain.nbr27)
                                        if i != 13 and r >= 0):
            self._setup_transport(transport or settings.transport)

    # ------------------------------------------------------------------------------------
    def _setup_transport(self, kind: str) -> None:
        kind = (kind or "auto").lower()
        if kind == "auto":
            chain = ["rccl", "torch", "host"] if self.backend == "hip" else ["torch"]
            if (self._skip_rccl or _RCCL_FAILED[0]) and self.backend == "hip":
                chain = ["torch", "host"]  # RCCL failed to set up earlier in this job
            errors = []
            for k in chain:
                try:
                    self._setup_transport(k)
                    # a transport can set up and still fail on first use (e.g. NCCL through
                    # torch with two ranks on one GPU): prove it with one exchange of the
                    # (not yet initialised) buffers -- ghost cells only, refilled by init
                    self.engine.exchange()
                    self.engine.sync()
                    ok = self.ctx.allreduce(1.0, "min") if self.ctx.is_distributed else 1.0
                except Exception as ex:  # pragma: no cover - exercised on multi-GPU nodes
                    errors.append(f"{k}: {ex}")
                    ok = self.ctx.allreduce(0.0, "min") if self.ctx.is_distributed else 0.0
                if ok <= 0:
                    if k == "rccl":
                        _RCCL_FAILED[0] = True
                    # a transport that set up but failed its trial (on any rank) must not stay
                    # behind the next one: abort its communicator / unmap its peers first
                    self.engine.drop_transport()
                    self.transport = "none"
                    self._torch_transport = None
                if ok > 0:
                    if errors and self.ctx.rank == 0:
                        import warnings
                        warnings.warn("halo transport fell back to " + k + " (" +
                                      "; ".join(errors) + ")")
                    return
            raise RuntimeError("no halo transport could be set up: " + "; ".join(errors))
        if kind == "rccl":
            if self.backend != "hip":
                raise ValueError("the rccl transport needs backend = AMDGPU/HIP")
            uid = native.rccl_unique_id() if self.ctx.rank == 0 else None
            uid = self.ctx.broadcast_object(uid, src=0)
            self.engine.rccl_init(uid, self.ctx.world_size, self.ctx.rank)
        elif kind == "ipc":
            # direct peer writes into the neighbours' landing buffers over xGMI, ordered by
            # device-side sequence flags (HipBackend::ipc_export / ipc_connect)
            if self.backend != "hip":
                raise ValueError("the ipc transport needs backend = AMDGPU/HIP")
            # every rank runs the same collectives whatever fails locally, then all agree: a
            # rank that cannot export or map must not leave its peers in a collective it skips
            err = None
            try:
                h = self.engine.ipc_export(self.ctx.world_size, self.ctx.rank)
            except Exception as ex:  # pragma: no cover - GPU-only failure path
                err, h = ex, b""
            plan = self.engine.plan()
            mine = (plan["recv_cells"], [(m["peer"], m["offset"], m["cells"]) for m in plan["recv"]])
            handles = self.ctx.allgather_object(h)
            tables = self.ctx.allgather_object(mine)
            if err is None and all(handles):
                try:
                    self.engine.ipc_connect(handles, tables)
                except Exception as ex:  # pragma: no cover - GPU-only failure path
                    err = ex
            elif err is None:
                err = RuntimeError("a peer could not export its IPC buffers")
            # also: no rank stores into a peer's landing buffer before every rank has mapped
            if self.ctx.allreduce(0.0 if err else 1.0, "min") <= 0:
                raise RuntimeError(f"ipc transport set-up failed on some rank: {err}")
            # gated passes (gate.hpp) on every rank or on none: a rank whose sub-domain cannot
            # run them (too few planes, a peer it cannot map) keeps the stream-overlapped passes,
            # and so must every peer -- the tuning passes and exchange counts must match
            if self.ctx.is_distributed:
                _agree_gated_depths(self.engine, self.ctx, self.fuse)
        elif kind in ("torch", "host"):
            stage = kind == "host" and self.backend == "hip"
            group = self.ctx.nccl_group() if (self.backend == "hip" and not stage) else None
            self._torch_transport = TorchTransport(self.engine.plan(), self.sendbuf, self.recvbuf,
                                                   self.domain.rank, group, stage_host=stage)
            self.engine.set_transport(self._torch_transport)
        else:
            raise ValueError(f"unknown transport {kind!r}")
        self.transport = kind

    def device_info(self) -> dict:
        """Where this rank runs and what its halo transport sees (bench.py's ``world``)."""
        info = {"rank": self.domain.rank, "backend": self.backend, "transport": self.transport}
        if self.backend == "hip":
            info["device"] = int(self.device.index)
            info["pci"] = native.device_pci_bus_id()
            rc = self.engine.rccl_info()
            if rc is not None:
                info["rccl_nranks"], info["rccl_rank"], info["rccl_device"] = rc
            if self.transport == "ipc":
                # which peers this rank maps, the device each runs on (as numbered here) and
                # whether hipDeviceCanAccessPeer confirmed the path (-1: not checkable)
                info["ipc_peers"] = [{"rank": r, "device": d, "peer_access": a}
                                     for r, d, a in self.engine.ipc_peers()]
        return info

    @property
    def overlapped(self) -> bool:
        """Whether full-depth passes overlap their halo exchange with the update: gated (the
        exchange inside the pass's fused launch) or stream-overlapped (inner part + shell)."""
        return self.engine.gated(self.fuse) or self.engine.overlapped(self.fuse)

    @property
    def gated(self) -> bool:
        """Whether full-depth passes carry the halo exchange inside their fused launch (the IPC
        transport, csrc/hip/gate.hpp): pack, signal, wait and unpack in the kernel."""
        return self.engine.gated(self.fuse)

    @property
    def depth(self) -> int:
        """Steps per pass (per halo exchange): ``fuse``, or -- single rank, after
        init_fields -- the depth <= fuse with the lowest measured kernel time per step."""
        return self.engine.depth()

    # ------------------------------------------------------------------------------------
    def init_fields(self) -> None:
        self.engine.init_fields()
        # pick the fastest fused-kernel tile/schedule on this device for this sub-domain
        # (timed on the live buffers; the state is unchanged) before any timed stepping
        self.engine.prepare()

    def fused_choice(self):
        """{depth: (config, schedule, ms)} chosen by the on-device autotuner (HIP only)."""
        if self.backend != "hip":
            return {}
        out = {}
        for n in range(2, self.fuse + 1):
            c = self.engine.fused_choice(n)
            if c is not None:
                out[n] = c
        return out

    def iterate(self, nsteps: int = 1) -> None:
        """Advance ``nsteps`` steps (each = exchange! + calculate! + swap in the reference)."""
        if nsteps > 0:
            self.engine.advance(nsteps)

    def halo_bytes(self) -> dict:
        """Bytes this rank sends to each neighbour rank per halo exchange (every message of the
        plan: faces, and with H > 1 edges and corners; z-plane plans send whole padded
        planes)."""
        itemsize = 4 if self.dtype == "float32" else 8
        out = {}
        for m in self.engine.plan()["send"]:
            if m["peer"] == self.domain.rank and self.transport == "none":
                continue  # periodic wrap onto this rank: a device copy, not a link
            out[m["peer"]] = out.get(m["peer"], 0) + 2 * itemsize * m["cells"]
        return out

    def phase_profile(self, steps: int) -> dict:
        """Advance ``steps`` steps with every phase of every pass timed in stream order on the
        device (csrc/include/gs/phase.h): median microseconds per pass of pack,
        transport, unpack, inner, shell, fused, step and bc, the halo exchange's span and the
        window's time per pass.  Derived: ``critical_us`` -- the pass's critical path from the
        parts (one overlapped pass: max(inner, exchange) + shell; chained overlapped passes,
        engine.h advance_chained, whose shell of pass p runs beside the inner part of pass p:
        the steady-state period max(inner, exchange + shell); otherwise the sum; plus bc
        weighted by the share of passes that refill the boundary) -- and
        ``accounted`` = critical_us / pass_us; ``bytes_per_neighbour`` and the achieved
        ``link_GBps`` (bytes to the busiest neighbour / the exchange's data time: transport, plus
        the pack for IPC, whose pack kernel stores straight into the peers)."""
        depth = max(1, int(self.depth))
        passes = max(1, -(-int(steps) // depth))
        self.engine.prof_start(64 * passes + 16)
        try:
            self.engine.advance(int(steps))
        finally:
            r = self.engine.prof_stop()
        chained = passes >= 2 and self.engine.chained(depth)
        crit = critical_path(r["phase_us"], r["exchange_us"], r["per_pass"], chained)
        r["critical_us"] = crit
        r["accounted"] = crit / r["pass_us"] if r["pass_us"] > 0 else None
        nb = self.halo_bytes()
        r["bytes_per_neighbour"] = {str(k): v for k, v in sorted(nb.items())}
        ph = r["phase_us"]
        data_us = ph.get("transport", 0.0) + (ph.get("pack", 0.0) if self.transport == "ipc" else 0.0)
        r["link_GBps"] = (float(f"{max(nb.values()) / (data_us * 1e3):.4g}")
                          if nb and data_us > 0 else None)
        r["transport"] = self.transport
        r["overlapped"] = bool(self.overlapped)
        # gated passes: the exchange runs inside the "fused" phase (one launch per pass)
        r["gated"] = bool(self.gated)
        if r["gated"]:
            r["gate"] = self.engine.gate_info(depth)
        r["chained"] = bool(chained)
        r["depth"] = depth
        return r

    @property
    def step(self) -> int:
        return self.engine.step

    def set_step(self, t: int) -> None:
        self.engine.set_step(t)

    def synchronize(self) -> None:
        self.engine.sync()

    def exchange(self) -> None:
        self.engine.exchange()

    # ------------------------------------------------------------------------------------
    @property
    def local_shape(self) -> Tuple[int, int, int]:
        """(nz, ny, nx): C-order shape of ghost-free local arrays (= Julia (x,y,z) column-major)."""
        nx, ny, nz = self.domain.proc_sizes
        return (nz, ny, nx)

    def get_fields_device(self) -> Tuple[torch.Tensor, torch.Tensor]:
        """Ghost-stripped copies of u, v on the field device (interior compaction kernel)."""
        tdt = _TORCH_DTYPES[self.dtype]
        u = torch.empty(self.local_shape, dtype=tdt, device=self.device)
        v = torch.empty(self.local_shape, dtype=tdt, device=self.device)
        self.engine.extract(u.data_ptr(), v.data_ptr())
        return u, v

    def get_fields(self) -> Tuple[np.ndarray, np.ndarray]:
        """Ghost-stripped host copies of u, v as (nz, ny, nx) numpy arrays."""
        if self.backend == "hip":
            # through the cached pinned snapshot buffers (one DMA per field), then host copies
            # the caller owns: a pageable .cpu() of a 512^3 field is staged in ~1 MB pieces
            # (~1 GB/s, 0.9 s per L=512 state in the bench's golden check)
            hu, hv, wait = self.snapshot_fields("get")
            wait()
            return hu.copy(), hv.copy()
        u, v = self.get_fields_device()
        return u.numpy(), v.numpy()

    _MM_CAP = 2048  # partial min / max quadruples of the snapshot kernel (kernels.hpp kMinMaxRows)

    def snapshot_fields(self, slot: str = "output", depth: int = 1, minmax: bool = False):
        """Asynchronous ghost-stripped copy of u, v for output: the compaction
        kernel runs in stream order on the compute stream, the D2H copy into pinned host
        buffers on a separate I/O stream, so stepping continues while the copy (and the file
        write that follows it) is in flight.  Returns ``(u, v, wait)``: numpy views of the host
        buffers and a callable that blocks until they are filled.

        Each ``slot`` (one per consumer: "output", "checkpoint") has one pair of device buffers
        and a ring of ``depth`` host buffer pairs, used in turn: the consumer must be done with
        a snapshot (its write joined) before the ``depth``-th next call of the same slot reuses
        its host buffers (the output stream keeps up to ``depth`` steps in flight).  The device
        buffers are not overwritten before the previous D2H copy out of them has finished (the
        compute stream waits for it), so consumers of different slots never race.

        ``minmax``: also return, as a fourth element, a callable giving ((u min, u max), (v min,
        v max)) of the snapshot once ``wait()`` has returned -- computed by the snapshot kernel
        itself (per-chunk partials copied with the data), so the BP4 writer need not scan the
        arrays for its block characteristics."""
        if self.backend != "hip":
            u, v = self.get_fields()
            if minmax:
                return u, v, lambda: None, lambda: ((u.min(), u.max()), (v.min(), v.max()))
            return u, v, lambda: None
        tdt = _TORCH_DTYPES[self.dtype]
        depth = max(1, int(depth))
        if getattr(self, "_snaps", None) is None:
            self._snaps = {}
            self._io_stream = torch.cuda.Stream(self.device)
        st = self._snaps.get(slot)
        if st is None or len(st["host"]) != depth:
            if st is not None and st["done"] is not None:
                st["done"].synchronize()  # the old ring's last copy has landed
            cap = self._MM_CAP
            st = self._snaps[slot] = {
                "dev": [torch.empty(self.local_shape, dtype=tdt, device=self.device)
                        for _ in range(2)] + [torch.empty(4 * cap, dtype=tdt, device=self.device)],
                "host": [[torch.empty(self.local_shape, dtype=tdt, pin_memory=True)
                          for _ in range(2)] + [torch.empty(4 * cap, dtype=tdt, pin_memory=True)]
                         for _ in range(depth)],
                "next": 0, "done": None}
        dev, host = st["dev"], st["host"][st["next"]]
        st["next"] = (st["next"] + 1) % depth
        # one native call (HipBackend::snapshot): the compute stream waits for the previous D2H
        # out of dev[] (event "done" of the last call), compacts (+ min / max partials), the I/O
        # stream copies into the pinned ring slot -- ~10 us of host time instead of the ~60-190
        # us of separate torch stream / event / copy calls
        if not self.native_snapshot:
            return self._snapshot_torch(st, dev, host, minmax)
        evs = st.setdefault("events", [])
        if len(evs) < 2 * depth + 2:
            evs.extend(native.NativeEvent() for _ in range(2 * depth + 2 - len(evs)))
        k = st.setdefault("ev_next", 0)
        st["ev_next"] = (k + 2) % len(evs)
        ready, done = evs[k], evs[k + 1]
        nmm = self.engine.snapshot(dev[0].data_ptr(), dev[1].data_ptr(),
                                   dev[2].data_ptr() if minmax else 0, self._MM_CAP,
                                   host[0].data_ptr(), host[1].data_ptr(),
                                   host[2].data_ptr() if minmax else 0,
                                   self._io_stream.cuda_stream, st["done"], ready, done)
        st["done"] = done
        return self._snapshot_views(host, nmm, done, minmax)

    # the snapshot through torch stream / event / copy calls (A/B of the native call:
    # scripts/profile_output.py --torch-snapshot)
    native_snapshot = True

    def prepare_snapshots(self, slot: str, depth: int = 1, minmax: bool = False) -> None:
        """Allocate ``slot``'s snapshot ring and fill every ring slot once (then wait): the
        state is unchanged; later snapshots of that slot start from warm buffers."""
        if self.backend != "hip":
            return
        wait = None
        for _ in range(max(1, int(depth))):
            wait = self.snapshot_fields(slot, depth=depth, minmax=minmax)[2]
        wait()

    def _snapshot_torch(self, st, dev, host, minmax):
        cur = torch.cuda.current_stream(self.device)
        if st["done"] is not None:
            cur.wait_event(st["done"])  # the previous D2H out of dev[] has finished
        nmm = 0
        if minmax:
            nmm = self.engine.extract_minmax(dev[0].data_ptr(), dev[1].data_ptr(),
                                             dev[2].data_ptr(), self._MM_CAP)
        if not nmm:
            self.engine.extract(dev[0].data_ptr(), dev[1].data_ptr())
        ready = torch.cuda.Event()
        ready.record(cur)
        done = torch.cuda.Event()
        with torch.cuda.stream(self._io_stream):
            self._io_stream.wait_event(ready)
            host[0].copy_(dev[0], non_blocking=True)
            host[1].copy_(dev[1], non_blocking=True)
            if nmm:
                host[2][:4 * nmm].copy_(dev[2][:4 * nmm], non_blocking=True)
            done.record(self._io_stream)
        st["done"] = done
        return self._snapshot_views(host, nmm, done, minmax)

    def _snapshot_views(self, host, nmm, done, minmax):
        u, v = host[0].numpy(), host[1].numpy()
        if not minmax:
            return u, v, done.synchronize
        part = host[2].numpy()[:4 * nmm].reshape(nmm, 4) if nmm else None
        if nmm:
            def mm():
                return ((part[:, 0].min(), part[:, 1].max()), (part[:, 2].min(), part[:, 3].max()))
        else:
            def mm():
                return ((u.min(), u.max()), (v.min(), v.max()))
        mm.part = part  # the raw quadruples (io/output.py hands them to the native writer)
        return u, v, done.synchronize, mm

    def set_fields(self, u, v) -> None:
        """Overwrite the interior of the current state (restart).  ``u``, ``v``: (nz, ny, nx)
        numpy arrays or torch tensors (any device)."""
        tdt = _TORCH_DTYPES[self.dtype]

        def dev(a):
            a = a if isinstance(a, torch.Tensor) else torch.as_tensor(np.ascontiguousarray(a))
            return a.to(device=self.device, dtype=tdt).contiguous()

        tu, tv = dev(u), dev(v)
        if tuple(tu.shape) != self.local_shape or tuple(tv.shape) != self.local_shape:
            raise ValueError(f"expected local arrays of shape {self.local_shape}")
        self.engine.insert(tu.data_ptr(), tv.data_ptr())
        self.engine.sync()

    def randomize_fields(self, seed: int = 0, lo: float = 0.0, hi: float = 1.0) -> None:
        """Random-init the interior: u, v ~ U[lo, hi) (benchmarks on "random-init u/v fields",
        BASELINE.json), drawn in place by the native engine from a counter-based Philox stream
        keyed on the *global* cell id (gs::random_init_cell): every decomposition -- and the
        golden model on any sub-box -- starts from the same global state."""
        self.engine.randomize(seed, lo, hi)
        self.engine.sync()

    def full_state(self, which: Optional[int] = None) -> torch.Tensor:
        """View of a raw state buffer as (pz, py, px, 2) including ghosts and padding."""
        g = self.geom
        b = self.buffers[self.engine.current if which is None else which]
        return b.view(g.pz, g.py, g.px, 2)

    def poison_ghosts(self, value: float = float("nan")) -> None:
        """Debug aid (SURVEY.md §5.2 halo poisoning): overwrite every non-interior cell of both
        buffers -- ghost shells, row padding, neighbour halos -- with ``value`` and forget the
        outer-boundary ghost parity.  A correct exchange / boundary refresh never lets the
        poison reach the interior, so a following run must equal an unpoisoned one."""
        g = self.geom
        H, xo = g.H, g.xo
        nx, ny, nz = self.domain.proc_sizes
        self.engine.sync()
        for b in self.buffers:
            full = b.view(g.pz, g.py, g.px, 2)
            keep = full[H:H + nz, H:H + ny, xo:xo + nx].clone()
            full.fill_(value)
            full[H:H + nz, H:H + ny, xo:xo + nx] = keep
        if self.backend == "hip":
            torch.cuda.synchronize(self.device)
        self.engine.set_step(self.engine.step)  # outer ghosts are refilled before next use

    def stats(self):
        """Local [sum_u, min_u, max_u, sum_v, min_v, max_v]."""
        return self.engine.stats()

    def global_stats(self):
        s = self.stats()
        tot = self.ctx.allreduce_array([s[0], s[3]], "sum")
        mn = self.ctx.allreduce_array([s[1], s[4]], "min")
        mx = self.ctx.allreduce_array([s[2], s[5]], "max")
        n = float(np.prod(self.domain.L))
        return {"mean_u": tot[0] / n, "min_u": mn[0], "max_u": mx[0],
                "mean_v": tot[1] / n, "min_v": mn[1], "max_v": mx[1]}

    def close(self, barrier: bool = True) -> None:
        """Free the engine.  With the IPC transport every rank drains its streams and meets the
        others at a barrier first (peers store into this rank's landing buffer until their last
        exchange); ``barrier=False``: the caller has already done both on every rank."""
        if getattr(self, "_snaps", None):
            self._io_stream.synchronize()  # no D2H copy may still read the snapshot buffers
            self._snaps = None
        if getattr(self, "engine", None) is not None:
            if self.transport == "ipc" and barrier:
                # peers store into this rank's landing buffer and flags until their last
                # exchange has finished: every rank drains its streams before any rank frees
                try:
                    self.engine.sync()
                finally:
                    self.ctx.barrier()
            self.engine.close()
            self.engine = None
