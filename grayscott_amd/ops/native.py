"""ctypes bindings to the native libraries built from ``csrc/``.

* ``libgs_core.so`` -- CPU/OpenMP backend (golden model) + shared scheduler
* ``libgs_hip.so``  -- gfx950 HIP kernels + RCCL halo transport + the same scheduler

Both export the C ABI of ``csrc/include/gs/capi.h``.  There is deliberately no silent
fallback: asking for the HIP backend when ``libgs_hip.so`` is missing raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
from ctypes import (CFUNCTYPE, POINTER, Structure, byref, c_char_p, c_double, c_int, c_int32,
                    c_int64, c_uint32, c_uint64, c_void_p)
from typing import Optional

_LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib")

DTYPE_CODES = {"float32": 0, "float64": 1}


class Geom(Structure):
    _fields_ = [
        ("nx", c_int32), ("ny", c_int32), ("nz", c_int32), ("H", c_int32),
        ("xo", c_int32), ("px", c_int32), ("py", c_int32), ("pz", c_int32),
        ("ox", c_int64), ("oy", c_int64), ("oz", c_int64),
        ("Lx", c_int64), ("Ly", c_int64), ("Lz", c_int64),
        ("periodic", c_int32), ("_pad", c_int32),
    ]


class Params(Structure):
    _fields_ = [
        ("F", c_double), ("k", c_double), ("dt", c_double), ("Du", c_double), ("Dv", c_double),
        ("noise", c_double), ("seed", c_uint64),
    ]


TRANSPORT_FN = CFUNCTYPE(c_int, c_void_p)

_libs = {}
_lock = threading.Lock()


class NativeLibraryMissing(RuntimeError):
    pass


def lib_path(name: str) -> str:
    """``libgs_<name>.so``; GS_HIP_VARIANT=abl selects the ablation build of the HIP library
    (``make ablation``: timing experiments only, its ablation kernels compute wrong results)."""
    if name == "hip" and os.environ.get("GS_HIP_VARIANT", "") == "abl":
        return os.path.join(_LIB_DIR, "libgs_hip_abl.so")
    return os.path.join(_LIB_DIR, f"libgs_{name}.so")


def _declare(lib) -> None:
    lib.gs_create.restype = c_void_p
    lib.gs_create.argtypes = [c_int32, POINTER(Geom), POINTER(Params), POINTER(c_int32), c_int32,
                              c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]
    lib.gs_destroy.argtypes = [c_void_p]
    lib.gs_destroy.restype = None
    lib.gs_last_error.restype = c_char_p
    for name in ("gs_init_fields", "gs_prepare", "gs_exchange", "gs_current_buffer", "gs_sync"):
        getattr(lib, name).argtypes = [c_void_p]
        getattr(lib, name).restype = c_int
    lib.gs_advance.argtypes = [c_void_p, c_int64]
    lib.gs_advance.restype = c_int
    lib.gs_plan_zplanes.argtypes = [c_void_p]
    lib.gs_plan_zplanes.restype = c_int
    lib.gs_set_overlap.argtypes = [c_void_p, c_int32]
    lib.gs_set_overlap.restype = c_int
    lib.gs_set_loopback.argtypes = [c_void_p, c_int32]
    lib.gs_set_loopback.restype = c_int
    lib.gs_overlapped.argtypes = [c_void_p, c_int32]
    lib.gs_overlapped.restype = c_int
    lib.gs_chained.argtypes = [c_void_p, c_int32]
    lib.gs_chained.restype = c_int
    lib.gs_gated.argtypes = [c_void_p, c_int32]
    lib.gs_gated.restype = c_int
    if hasattr(lib, "gs_snapshot"):
        lib.gs_snapshot.argtypes = [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_int32,
                                    c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p]
        lib.gs_snapshot.restype = c_int
    lib.gs_set_gated.argtypes = [c_void_p, c_int32]
    lib.gs_set_gated.restype = c_int
    lib.gs_depth.argtypes = [c_void_p]
    lib.gs_depth.restype = c_int
    lib.gs_set_auto_depth.argtypes = [c_void_p, c_int32]
    lib.gs_set_auto_depth.restype = c_int
    lib.gs_get_step.argtypes = [c_void_p]
    lib.gs_get_step.restype = c_int64
    lib.gs_set_step.argtypes = [c_void_p, c_int64]
    lib.gs_set_step.restype = c_int
    lib.gs_extract.argtypes = [c_void_p, c_void_p, c_void_p]
    lib.gs_extract.restype = c_int
    lib.gs_extract_minmax.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int32]
    lib.gs_extract_minmax.restype = c_int
    lib.gs_insert.argtypes = [c_void_p, c_void_p, c_void_p]
    lib.gs_insert.restype = c_int
    lib.gs_stats.argtypes = [c_void_p, POINTER(c_double)]
    lib.gs_stats.restype = c_int
    lib.gs_randomize.argtypes = [c_void_p, c_uint64, c_double, c_double]
    lib.gs_randomize.restype = c_int
    lib.gs_drop_transport.argtypes = [c_void_p]
    lib.gs_drop_transport.restype = c_int
    lib.gs_set_transport.argtypes = [c_void_p, TRANSPORT_FN, c_void_p]
    lib.gs_set_transport.restype = c_int
    lib.gs_plan_info.argtypes = [c_void_p, POINTER(c_int64), POINTER(c_int64), POINTER(c_int32),
                                 POINTER(c_int32)]
    lib.gs_plan_info.restype = c_int
    lib.gs_plan_msg.argtypes = [c_void_p, c_int32, c_int32, POINTER(c_int64)]
    lib.gs_plan_msg.restype = c_int
    lib.gs_geom_total_elems.argtypes = [POINTER(Geom)]
    lib.gs_geom_total_elems.restype = c_int64
    lib.gs_make_geom.argtypes = [POINTER(Geom), c_int, c_int, c_int, c_int, c_int64, c_int64,
                                 c_int64, c_int64, c_int64, c_int64, c_int]
    lib.gs_make_geom.restype = None
    lib.gs_noise_block.argtypes = [c_int64, c_int64, c_int64, c_int64, c_int64, c_uint64, c_uint64,
                                   POINTER(c_uint32)]
    lib.gs_noise_block.restype = None
    lib.gs_plan_sizes.argtypes = [POINTER(Geom), POINTER(c_int32), c_int32, POINTER(c_int64),
                                  POINTER(c_int64)]
    lib.gs_plan_sizes.restype = c_int
    if hasattr(lib, "gs_rccl_unique_id"):
        lib.gs_rccl_unique_id.argtypes = [ctypes.c_char_p, c_int32]
        lib.gs_rccl_unique_id.restype = c_int
        lib.gs_rccl_init.argtypes = [c_void_p, ctypes.c_char_p, c_int32, c_int32, c_int32]
        lib.gs_rccl_init.restype = c_int
        lib.gs_rccl_info.argtypes = [c_void_p, c_int32, POINTER(c_int32)]
        lib.gs_rccl_info.restype = c_int
        lib.gs_rccl_abort.argtypes = []
        lib.gs_rccl_abort.restype = c_int
        lib.gs_device_pci.argtypes = [ctypes.c_char_p, c_int32]
        lib.gs_device_pci.restype = c_int
    if hasattr(lib, "gs_ipc_export"):
        lib.gs_ipc_handle_bytes.argtypes = []
        lib.gs_ipc_handle_bytes.restype = c_int
        lib.gs_ipc_tab_stride.argtypes = []
        lib.gs_ipc_tab_stride.restype = c_int
        lib.gs_ipc_export.argtypes = [c_void_p, c_int32, c_int32, c_int32, ctypes.c_char_p]
        lib.gs_ipc_export.restype = c_int
        lib.gs_ipc_connect.argtypes = [c_void_p, c_int32, ctypes.c_char_p, POINTER(c_int64)]
        lib.gs_ipc_connect.restype = c_int
        lib.gs_ipc_peers.argtypes = [c_void_p, c_int32, POINTER(c_int32), c_int32]
        lib.gs_ipc_peers.restype = c_int
    lib.gs_prof_len.argtypes = []
    lib.gs_prof_len.restype = c_int
    lib.gs_phase_count.argtypes = []
    lib.gs_phase_count.restype = c_int
    lib.gs_phase_name.argtypes = [c_int32]
    lib.gs_phase_name.restype = c_char_p
    lib.gs_prof_start.argtypes = [c_void_p, c_int32]
    lib.gs_prof_start.restype = c_int
    lib.gs_prof_stop.argtypes = [c_void_p, POINTER(c_double)]
    lib.gs_prof_stop.restype = c_int
    if hasattr(lib, "gs_peer_access"):
        lib.gs_peer_access.argtypes = [POINTER(c_int32), c_int32]
        lib.gs_peer_access.restype = c_int
    if hasattr(lib, "gs_fused_choice"):
        lib.gs_fused_choice.argtypes = [c_void_p, c_int32, c_int32, POINTER(c_int32),
                                        POINTER(ctypes.c_float)]
        lib.gs_fused_choice.restype = c_int


def load(name: str):
    """Load ``libgs_<name>.so`` ("core" or "hip"); raise if it was not built."""
    with _lock:
        if name in _libs:
            return _libs[name]
        path = lib_path(name)
        if not os.path.exists(path):
            raise NativeLibraryMissing(
                f"{path} not found: build the native libraries first (`make` or "
                f"`python -c 'import __graft_entry__ as g; g.build()'`)")
        lib = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
        _declare(lib)
        _libs[name] = lib
        return lib


def last_error(lib) -> str:
    msg = lib.gs_last_error()
    return msg.decode() if msg else "unknown error"


def check(lib, rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: {last_error(lib)}")


def make_geom(nx, ny, nz, H, ox, oy, oz, Lx, Ly, Lz, periodic) -> Geom:
    g = Geom()
    load("core").gs_make_geom(ctypes.byref(g), nx, ny, nz, H, ox, oy, oz, Lx, Ly, Lz,
                              1 if periodic else 0)
    return g


def total_elems(g: Geom) -> int:
    return int(load("core").gs_geom_total_elems(ctypes.byref(g)))


def plan_sizes(g: Geom, nbr27, diagonals: bool):
    arr = (c_int32 * 27)(*nbr27)
    s, r = c_int64(), c_int64()
    load("core").gs_plan_sizes(ctypes.byref(g), arr, 1 if diagonals else 0, ctypes.byref(s),
                               ctypes.byref(r))
    return int(s.value), int(r.value)


def gate_plan(g: Geom, nbr27, n: int, xp: int = 0, allpk: bool = False, slots: int = 256,
              longest: bool = False, rows: int = 4, waves: int = 12, fold: bool = False,
              pairs: bool = False, unpack: int = 0):
    """The gated pass's unit table for a sub-domain (csrc/include/gs/gate_plan.h, host only):
    ``(units, npk, grid)`` -- units as (tile, z0, z1, pk, wait, prod) tuples, the packer count and the
    tile grid {xstep, ystep, ybase, ntx, nty, ntxf, nfold, ntiles, rt}.  pairs: the
    two-units-per-workgroup table (entries 2w, 2w + 1; tile -1 = empty), xp the expected
    exchange and ``unpack`` the cone unpack, in plane-times."""
    lib = load("core")
    lib.gs_gate_plan.restype = c_int
    arr = (c_int32 * 27)(*nbr27)
    grid = (c_int32 * 9)()
    npk = c_int32()
    cap = 1 << 16
    out = (c_int32 * (6 * cap))()
    k = lib.gs_gate_plan(ctypes.byref(g), arr, int(n), int(xp), 1 if allpk else 0, int(slots),
                         1 if longest else 0, int(rows), int(waves), 1 if fold else 0,
                         1 if pairs else 0, int(unpack), out, cap, ctypes.byref(npk), grid)
    if k < 0 or k > cap:
        raise ValueError(f"gs_gate_plan failed ({k})")
    units = [tuple(out[6 * i:6 * i + 6]) for i in range(k)]
    keys = ("xstep", "ystep", "ybase", "ntx", "nty", "ntxf", "nfold", "ntiles", "rt")
    return units, int(npk.value), dict(zip(keys, list(grid)))


def plan_depths(cost: dict, nsteps: int, fill: float = 0.0, pp: int = -1) -> list:
    """gs::plan_depths (engine.h): the cheapest partition of ``nsteps`` into fused passes of
    depth 2..max(cost), given each depth's pass time ``cost[k]``; deepest passes first.  With
    ``fill`` > 0 every depth-parity switch between consecutive passes costs one outer-ghost
    refresh of ``fill`` (``pp``: the parity a first pass needs to avoid one, -1 none), and the
    passes come grouped by parity."""
    lib = load("core")
    kmax = max(cost)
    arr = (c_double * 8)(*[float(cost.get(k, 0.0)) for k in range(8)])
    cap = 1 << 16
    out = (c_int32 * cap)()
    if fill > 0.0 or pp >= 0:
        lib.gs_plan_depths_bc.argtypes = [POINTER(c_double), c_int32, c_int64, c_double, c_int32,
                                          POINTER(c_int32), c_int32]
        lib.gs_plan_depths_bc.restype = c_int
        n = lib.gs_plan_depths_bc(arr, int(kmax), int(nsteps), float(fill), int(pp), out, cap)
    else:
        lib.gs_plan_depths.argtypes = [POINTER(c_double), c_int32, c_int64, POINTER(c_int32),
                                       c_int32]
        lib.gs_plan_depths.restype = c_int
        n = lib.gs_plan_depths(arr, int(kmax), int(nsteps), out, cap)
    if n < 0:
        raise ValueError("plan_depths: depths must be 2..7")
    return [int(out[i]) for i in range(min(n, cap))]


def noise_block(gx, gy, gz4, Lx, Ly, step, seed):
    out = (c_uint32 * 4)()
    load("core").gs_noise_block(gx, gy, gz4, Lx, Ly, step, seed, out)
    return [int(v) for v in out]


class Engine:
    """Thin owner of a native ``gs_engine`` handle."""

    def __init__(self, backend: str, dtype: str, geom: Geom, params: Params, nbr27, rank: int,
                 fuse: int, use_fused: bool, buf0: int, buf1: int, send: int, recv: int,
                 stream: int = 0):
        self.lib = load("hip" if backend == "hip" else "core")
        self.backend = backend
        self.dtype = dtype
        self._nbr = (c_int32 * 27)(*nbr27)
        self._geom = geom
        self._params = params
        h = self.lib.gs_create(DTYPE_CODES[dtype], ctypes.byref(geom), ctypes.byref(params),
                               self._nbr, rank, fuse, 1 if use_fused else 0, c_void_p(buf0),
                               c_void_p(buf1), c_void_p(send or None), c_void_p(recv or None),
                               c_void_p(stream or None))
        if not h:
            raise RuntimeError(f"gs_create failed: {last_error(self.lib)}")
        self.h = c_void_p(h)
        self._cb = None

    def close(self):
        if getattr(self, "h", None):
            self.lib.gs_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        check(self.lib, rc, what)

    def init_fields(self):
        self._chk(self.lib.gs_init_fields(self.h), "init_fields")

    def prepare(self):
        """Autotune the fused kernel on the live buffers (the state is left unchanged)."""
        self._chk(self.lib.gs_prepare(self.h), "prepare")

    def fused_choice(self, n: int):
        """(config name, schedule, ms) the autotuner picked for fuse depth n, or None."""
        if not hasattr(self.lib, "gs_fused_choice"):
            return None
        out = (c_int32 * 2)()
        ms = ctypes.c_float()
        self._chk(self.lib.gs_fused_choice(self.h, int(n), DTYPE_CODES[self.dtype], out,
                                           ctypes.byref(ms)), "fused_choice")
        if out[0] < 0:
            return None
        return fused_cfg_name(int(out[0])), int(out[1]), float(ms.value)

    def set_overlap(self, mode: int):
        """-1 auto, 0 off, 1 on (where the plan and backend allow it)."""
        self._chk(self.lib.gs_set_overlap(self.h, int(mode)), "set_overlap")

    def set_loopback(self, on: bool):
        """Send messages to this rank through the device transport too (single-GPU tests)."""
        self._chk(self.lib.gs_set_loopback(self.h, 1 if on else 0), "set_loopback")

    def overlapped(self, k: int) -> bool:
        return bool(self.lib.gs_overlapped(self.h, int(k)))

    def chained(self, k: int) -> bool:
        return bool(self.lib.gs_chained(self.h, int(k)))

    def gated(self, k: int) -> bool:
        """Whether k-step passes carry the halo exchange inside their fused launch (gate.hpp)."""
        return bool(self.lib.gs_gated(self.h, int(k)))

    def gate_stamps(self):
        """Debug knob gate_stamps: the last gated launch's exchange in µs after its first packer
        or waiting unit started -- {"packed" (-1: a carried exchange), "first_wait_done",
        "last_wait_done", "unpacked", one unit's unpack: "unit_unpack_max", "unit_unpack_mean",
        and over every launch since set-up one producer's carry: "carry_max", "carry_mean"
        (-1: none)}, or None."""
        if not hasattr(self.lib, "gs_gate_stamps"):
            return None
        out = (c_double * 8)()
        self.lib.gs_gate_stamps.argtypes = [c_void_p, c_int32, POINTER(c_double)]
        self.lib.gs_gate_stamps.restype = c_int
        if self.lib.gs_gate_stamps(self.h, DTYPE_CODES[self.dtype], out) != 0 or out[1] < 0:
            return None
        return dict(zip(("packed", "first_wait_done", "last_wait_done", "unpacked",
                         "unit_unpack_max", "unit_unpack_mean", "carry_max", "carry_mean"),
                        (round(float(x), 2) for x in out)))

    def set_gated(self, on: bool):
        """Allow / forbid gated passes on this engine (the job's ranks agree on it)."""
        self._chk(self.lib.gs_set_gated(self.h, 1 if on else 0), "set_gated")

    def set_gated_depth(self, k: int, on: bool):
        """Allow / forbid gated passes of depth k only (the ranks agree per depth)."""
        self.lib.gs_set_gated_depth.argtypes = [c_void_p, c_int32, c_int32]
        self.lib.gs_set_gated_depth.restype = c_int
        self._chk(self.lib.gs_set_gated_depth(self.h, int(k), 1 if on else 0), "set_gated_depth")

    def gate_info(self, k: int):
        """{"xp", "units" (workgroups), "packers", "ms", "pairs_unpack", "carried"} of the tuned
        gated pass of depth k (HIP only; pairs_unpack: the pairs table's U, None for a one-unit
        table; carried: the producers when runs of passes carry their exchanges, else None), or
        None."""
        if not hasattr(self.lib, "gs_gate_info"):
            return None
        out = (c_double * 6)()
        self.lib.gs_gate_info.argtypes = [c_void_p, c_int32, c_int32, POINTER(c_double)]
        self.lib.gs_gate_info.restype = c_int
        if self.lib.gs_gate_info(self.h, int(k), DTYPE_CODES[self.dtype], out) != 0 or out[0] < 0:
            return None
        pairs = out[4] >= 0
        return {"xp": int(out[0]), "units": int(out[1]) // (2 if pairs else 1),
                "packers": int(out[2]), "ms": round(float(out[3]), 5),
                "pairs_unpack": int(out[4]) if pairs else None,
                "carried": int(out[5]) if out[5] >= 0 else None}

    def set_auto_depth(self, on: bool):
        self._chk(self.lib.gs_set_auto_depth(self.h, 1 if on else 0), "set_auto_depth")

    def depth(self) -> int:
        """Steps per pass: the fuse depth, or the cheaper one measured by prepare()."""
        return int(self.lib.gs_depth(self.h))

    def set_plan(self, on: bool):
        """Pass-depth planner (engine.h plan_passes) on (default) or off (greedy schedule)."""
        self.lib.gs_set_plan.argtypes = [c_void_p, c_int32]
        self.lib.gs_set_plan.restype = c_int
        self._chk(self.lib.gs_set_plan(self.h, 1 if on else 0), "set_plan")

    def fill_ms(self) -> float:
        """One outer-ghost refresh as timed by prepare() (the planner's parity-switch cost)."""
        self.lib.gs_fill_ms.argtypes = [c_void_p]
        self.lib.gs_fill_ms.restype = c_double
        return float(self.lib.gs_fill_ms(self.h))

    def plan_passes(self, nsteps: int) -> list:
        """The pass depths advance(nsteps) runs ([] = the greedy min(nsteps, depth) schedule:
        multi-rank, an explicit fuse, or untimed depths)."""
        self.lib.gs_plan_passes.argtypes = [c_void_p, c_int64, POINTER(c_int32), c_int32]
        self.lib.gs_plan_passes.restype = c_int
        cap = 4096
        out = (c_int32 * cap)()
        n = self.lib.gs_plan_passes(self.h, int(nsteps), out, cap)
        if n < 0:
            self._chk(n, "plan_passes")
        return [int(out[i]) for i in range(min(n, cap))]

    def advance(self, n: int):
        self._chk(self.lib.gs_advance(self.h, int(n)), "advance")

    def exchange(self):
        self._chk(self.lib.gs_exchange(self.h), "exchange")

    @property
    def step(self) -> int:
        return int(self.lib.gs_get_step(self.h))

    def set_step(self, t: int):
        self._chk(self.lib.gs_set_step(self.h, int(t)), "set_step")

    @property
    def current(self) -> int:
        return int(self.lib.gs_current_buffer(self.h))

    def sync(self):
        self._chk(self.lib.gs_sync(self.h), "sync")

    def extract(self, u_ptr: int, v_ptr: int):
        self._chk(self.lib.gs_extract(self.h, c_void_p(u_ptr or None), c_void_p(v_ptr or None)),
                  "extract")

    def extract_minmax(self, u_ptr: int, v_ptr: int, part_ptr: int, cap: int) -> int:
        """extract() plus each chunk's (u min, u max, v min, v max) at ``part_ptr`` (``cap``
        quadruples of the field type): the number written, or 0 if the backend has no such
        path (the CPU backend)."""
        n = self.lib.gs_extract_minmax(self.h, c_void_p(u_ptr), c_void_p(v_ptr),
                                       c_void_p(part_ptr), int(cap))
        if n == -2:
            return 0
        self._chk(0 if n >= 0 else -1, "extract_minmax")
        return n

    def snapshot(self, du: int, dv: int, dpart: int, cap: int, hu: int, hv: int, hpart: int,
                 io_stream: int, prev, ready, done) -> int:
        """HIP only: compact the interior into (du, dv) [+ per-chunk min / max at dpart] on the
        compute stream after event ``prev``, copy to the pinned (hu, hv[, hpart]) on the I/O
        stream, record ``done`` (NativeEvent handles).  Returns the min / max quadruples."""
        n = self.lib.gs_snapshot(self.h, DTYPE_CODES[self.dtype], c_void_p(du), c_void_p(dv),
                                 c_void_p(dpart or None), int(cap), c_void_p(hu), c_void_p(hv),
                                 c_void_p(hpart or None), c_void_p(io_stream or None),
                                 c_void_p(prev.ptr if prev is not None else None),
                                 c_void_p(ready.ptr), c_void_p(done.ptr))
        self._chk(0 if n >= 0 else -1, "snapshot")
        return n

    def insert(self, u_ptr: int, v_ptr: int):
        self._chk(self.lib.gs_insert(self.h, c_void_p(u_ptr), c_void_p(v_ptr)), "insert")

    def randomize(self, seed: int, lo: float = 0.0, hi: float = 1.0):
        """Random interior, u, v ~ U[lo, hi): a function of the global cell and ``seed`` only
        (the same global state for every decomposition)."""
        self._chk(self.lib.gs_randomize(self.h, int(seed) & 0xFFFFFFFFFFFFFFFF, float(lo),
                                        float(hi)), "randomize")

    def drop_transport(self):
        """Forget the halo transport (abort the RCCL communicator, unmap IPC peers)."""
        self._chk(self.lib.gs_drop_transport(self.h), "drop_transport")

    def stats(self):
        out = (c_double * 6)()
        self._chk(self.lib.gs_stats(self.h, out), "stats")
        return list(out)

    def set_transport(self, fn):
        """``fn()`` -> None; exchanges send buffer into receive buffer (exceptions -> failure)."""

        def _tramp(_user):
            try:
                fn()
                return 0
            except Exception as ex:  # pragma: no cover - surfaced through last_error
                import traceback
                traceback.print_exc()
                return 1

        self._cb = TRANSPORT_FN(_tramp)
        self._chk(self.lib.gs_set_transport(self.h, self._cb, None), "set_transport")

    def plan(self):
        sc, rc = c_int64(), c_int64()
        ns, nr = c_int32(), c_int32()
        self.lib.gs_plan_info(self.h, ctypes.byref(sc), ctypes.byref(rc), ctypes.byref(ns),
                              ctypes.byref(nr))
        out = {"send_cells": sc.value, "recv_cells": rc.value, "send": [], "recv": [],
               "zplanes": bool(self.lib.gs_plan_zplanes(self.h))}
        buf = (c_int64 * 4)()
        for which, key, n in ((0, "send", ns.value), (1, "recv", nr.value)):
            for i in range(n):
                self.lib.gs_plan_msg(self.h, which, i, buf)
                out[key].append({"dir": int(buf[0]), "peer": int(buf[1]), "offset": int(buf[2]),
                                 "cells": int(buf[3])})
        return out

    def prof_start(self, max_records: int) -> None:
        """Open a per-phase timing window (csrc/include/gs/phase.h): every phase of every pass
        from now on is bracketed by timestamps in stream order (hipEvents on the GPU)."""
        self._chk(self.lib.gs_prof_start(self.h, int(max_records)), "prof_start")

    def prof_stop(self) -> dict:
        """Close the window: wait for the device, return the per-pass phase summary
        ``{"passes", "steps", "window_us", "pass_us", "exchange_us", "phase_us": {name: median
        us per pass}, "per_pass": {name: intervals per pass}, "truncated"}`` (phases that did not
        occur are left out)."""
        n = int(self.lib.gs_prof_len())
        out = (c_double * n)()
        rc = self.lib.gs_prof_stop(self.h, out)
        if rc < 0:
            raise RuntimeError(f"prof_stop failed: {last_error(self.lib)}")
        res = {"passes": int(out[0]), "steps": int(out[1]), "window_us": out[2],
               "pass_us": out[3], "exchange_us": out[4], "phase_us": {}, "per_pass": {},
               "truncated": bool(rc == 1)}
        for i in range(int(self.lib.gs_phase_count())):
            name = self.lib.gs_phase_name(i).decode()
            if out[6 + 2 * i] > 0:
                res["phase_us"][name] = out[5 + 2 * i]
                res["per_pass"][name] = out[6 + 2 * i]
        return res

    def rccl_init(self, uid: bytes, nranks: int, rank: int):
        if not hasattr(self.lib, "gs_rccl_init"):
            raise RuntimeError("RCCL transport needs the HIP backend")
        self._chk(self.lib.gs_rccl_init(self.h, uid, nranks, rank, DTYPE_CODES[self.dtype]),
                  "rccl_init")


    def ipc_export(self, nranks: int, rank: int) -> bytes:
        """IPC transport, step 1: allocate and export this engine's landing buffer and flags."""
        if not hasattr(self.lib, "gs_ipc_export"):
            raise RuntimeError("the IPC transport needs the HIP backend")
        buf = ctypes.create_string_buffer(int(self.lib.gs_ipc_handle_bytes()))
        n = self.lib.gs_ipc_export(self.h, DTYPE_CODES[self.dtype], int(nranks), int(rank), buf)
        if n < 0:
            raise RuntimeError(f"ipc_export failed: {last_error(self.lib)}")
        return buf.raw[:n]

    def ipc_connect(self, handles, recv_tables) -> None:
        """IPC transport, step 2: map the neighbours' exports.  ``handles[r]``: rank r's
        ``ipc_export`` bytes; ``recv_tables[r]``: (recv_cells, [(peer, offset, cells), ...]) of
        rank r's halo plan."""
        stride = int(self.lib.gs_ipc_tab_stride())
        tab = (c_int64 * (stride * len(handles)))()
        for r, (rcells, msgs) in enumerate(recv_tables):
            base = r * stride
            tab[base], tab[base + 1] = len(msgs), int(rcells)
            for j, (peer, off, cells) in enumerate(msgs):
                tab[base + 2 + 3 * j:base + 5 + 3 * j] = [int(peer), int(off), int(cells)]
        self._chk(self.lib.gs_ipc_connect(self.h, DTYPE_CODES[self.dtype], b"".join(handles), tab),
                  "ipc_connect")

    def ipc_peers(self):
        """[(peer rank, device as numbered here or -1, peer access 1 / -1 unknown)] of the IPC
        transport's mapped peers ([] without it)."""
        if not hasattr(self.lib, "gs_ipc_peers"):
            return []
        out = (c_int32 * (3 * 26))()
        n = self.lib.gs_ipc_peers(self.h, DTYPE_CODES[self.dtype], out, 26)
        if n < 0:
            raise RuntimeError(f"ipc_peers failed: {last_error(self.lib)}")
        return [(int(out[3 * i]), int(out[3 * i + 1]), int(out[3 * i + 2])) for i in range(n)]

    def rccl_info(self):
        """(communicator size, rank in it, HIP device) of the RCCL transport, or None."""
        if not hasattr(self.lib, "gs_rccl_info"):
            return None
        out = (c_int32 * 3)()
        self._chk(self.lib.gs_rccl_info(self.h, DTYPE_CODES[self.dtype], out), "rccl_info")
        return None if out[0] < 0 else (int(out[0]), int(out[1]), int(out[2]))


def rccl_abort() -> None:
    """Abort this process's RCCL communicator, if the HIP library is loaded and holds one."""
    lib = _libs.get("hip")
    if lib is not None and hasattr(lib, "gs_rccl_abort"):
        lib.gs_rccl_abort()


def device_pci_bus_id() -> str:
    """PCI bus id of the current HIP device ("" when unavailable)."""
    lib = load("hip")
    buf = ctypes.create_string_buffer(64)
    n = lib.gs_device_pci(buf, 64)
    return buf.value.decode() if n > 0 else ""


def peer_access_matrix():
    """hipDeviceCanAccessPeer for every pair of the devices this process sees: an n x n list
    of 1 / 0 (-1: the query failed); [] without the HIP library."""
    lib = load("hip")
    if not hasattr(lib, "gs_peer_access"):
        return []
    buf = (c_int32 * (64 * 64))()
    n = lib.gs_peer_access(buf, 64 * 64)
    if n < 0:
        return []
    return [[int(buf[i * n + j]) for j in range(n)] for i in range(n)]


def noise_blocks(q, step: int, seed: int, impl: int = -1):
    """Philox4x32-10 blocks of counters ``q`` (uint64: (q, q >> 32, step, step >> 32), key
    ``seed``) as an (n, 4) uint32 array, by the CPU backend's row routine: ``impl`` 0 scalar,
    1 AVX2 (None when the CPU lacks it), -1 the form its step uses."""
    import numpy as np
    lib = load("core")
    lib.gs_noise_blocks.argtypes = [c_void_p, c_int32, ctypes.c_uint64, ctypes.c_uint64,
                                    c_void_p, c_int32]
    lib.gs_noise_blocks.restype = c_int
    qa = np.ascontiguousarray(np.asarray(q, dtype=np.uint64))
    out = np.zeros((qa.size, 4), dtype=np.uint32)
    rc = lib.gs_noise_blocks(qa.ctypes.data, qa.size, int(step), int(seed), out.ctypes.data,
                             int(impl))
    return None if rc != 0 else out


def cpu_threads(n: int = 0) -> int:
    """OpenMP threads of the CPU backend in this process: ``n > 0`` sets them; returns the
    current maximum."""
    lib = load("core")
    lib.gs_cpu_threads.argtypes = [c_int32]
    lib.gs_cpu_threads.restype = c_int
    return int(lib.gs_cpu_threads(int(n)))


class NativeEvent:
    """A HIP event owned by Python (gs_event_create): ``synchronize()`` waits with the GIL
    released; destroyed with the object."""

    def __init__(self):
        self.lib = load("hip")
        self.lib.gs_event_create.restype = c_void_p
        self.lib.gs_event_destroy.argtypes = [c_void_p]
        self.lib.gs_event_sync.argtypes = [c_void_p]
        self.lib.gs_event_sync.restype = c_int
        self.ptr = self.lib.gs_event_create()
        if not self.ptr:
            raise RuntimeError("gs_event_create failed")

    def synchronize(self) -> None:
        if self.lib.gs_event_sync(self.ptr) != 0:
            raise RuntimeError(self.lib.gs_last_error().decode())

    def __del__(self):
        ptr, self.ptr = getattr(self, "ptr", None), None
        if ptr:
            try:
                self.lib.gs_event_destroy(ptr)
            except Exception:  # pragma: no cover - interpreter teardown
                pass


def debug_set(name: str, value: float, which: str = "hip") -> None:
    """Set a test / modelling switch of a native library (csrc/include/gs/debug.h):
    ``overlap_chain`` (0: overlapped passes one at a time; read at engine creation),
    ``philox_generic`` (1: the 64-bit-counter Philox path), ``ipc_emulate_us`` (minimum IPC
    exchange time).  Process-wide; never read from the environment."""
    lib = load(which)
    lib.gs_debug_set.argtypes = [ctypes.c_char_p, c_double]
    lib.gs_debug_set.restype = c_int
    if lib.gs_debug_set(name.encode(), float(value)) != 0:
        raise ValueError(f"unknown debug switch {name!r}")


def rccl_unique_id() -> bytes:
    lib = load("hip")
    buf = ctypes.create_string_buffer(256)
    n = lib.gs_rccl_unique_id(buf, 256)
    if n < 0:
        raise RuntimeError(f"ncclGetUniqueId failed: {last_error(lib)}")
    return buf.raw[:n]


def fused_select(name: str = "") -> None:
    """Pick a fused-kernel tuning configuration for fp32 ("" = measured default)."""
    lib = load("hip")
    lib.gs_fused_select.argtypes = [ctypes.c_char_p]
    lib.gs_fused_select.restype = c_int
    if lib.gs_fused_select(name.encode()) != 0:
        raise ValueError(f"unknown fused-kernel configuration {name!r}")


def fused_sched(sched: int) -> None:
    """Pick the fused-kernel work schedule: 0 even split, 1 XCD-grouped lockstep chunks (one
    per workgroup), 2 XCD-grouped chunks swept in rounds by a persistent grid."""
    lib = load("hip")
    lib.gs_fused_sched.argtypes = [c_int32]
    lib.gs_fused_sched.restype = c_int
    if lib.gs_fused_sched(int(sched)) != 0:
        raise ValueError(f"unknown schedule {sched}")


def fused_unpin() -> None:
    """Undo fused_select / fused_sched: engines created afterwards use the autotuner again."""
    lib = load("hip")
    lib.gs_fused_unpin.argtypes = []
    lib.gs_fused_unpin.restype = c_int
    lib.gs_fused_unpin()


def fused_cfg_lookup(name: str) -> int:
    """Index of fused-kernel configuration ``name`` in the loaded HIP library, -1 if this build
    does not have it (the ablation variants exist only in ``make ablation`` builds)."""
    lib = load("hip")
    lib.gs_fused_cfg_lookup.argtypes = [ctypes.c_char_p]
    lib.gs_fused_cfg_lookup.restype = c_int
    return int(lib.gs_fused_cfg_lookup(name.encode()))


def fused_cfg_name(index: int) -> str:
    """Name of fused-kernel configuration ``index`` ("" = measured default)."""
    lib = load("hip")
    lib.gs_fused_cfg_name.argtypes = [c_int32]
    lib.gs_fused_cfg_name.restype = c_char_p
    r = lib.gs_fused_cfg_name(int(index))
    return r.decode() if r is not None else f"#{index}"


class LinkProbe:
    """The link probe's device buffers (csrc/hip/probe.hpp): IPC peer-store puts and RCCL
    send / receive pairs, timed on the device.  ``nbytes``: the largest message it times."""

    def __init__(self, nbytes: int):
        lib = self.lib = load("hip")
        lib.gs_probe_create.argtypes = [ctypes.c_int64]
        lib.gs_probe_create.restype = c_void_p
        lib.gs_probe_destroy.argtypes = [c_void_p]
        lib.gs_probe_export.argtypes = [c_void_p, ctypes.c_char_p]
        lib.gs_probe_export.restype = c_int
        lib.gs_probe_ipc.argtypes = [c_void_p, ctypes.c_char_p, ctypes.c_int64, c_int32,
                                     POINTER(c_double)]
        lib.gs_probe_ipc.restype = c_int
        lib.gs_probe_rccl_init.argtypes = [c_void_p, ctypes.c_char_p, c_int32, c_int32]
        lib.gs_probe_rccl_init.restype = c_int
        lib.gs_probe_rccl.argtypes = [c_void_p, c_int32, ctypes.c_int64, c_int32,
                                      POINTER(c_double)]
        lib.gs_probe_rccl.restype = c_int
        self.h = lib.gs_probe_create(int(nbytes))
        if not self.h:
            raise RuntimeError(f"link probe: {last_error(lib)}")

    def export(self) -> bytes:
        buf = ctypes.create_string_buffer(512)
        n = self.lib.gs_probe_export(self.h, buf)
        if n < 0:
            raise RuntimeError(f"link probe export: {last_error(self.lib)}")
        return buf.raw[:n]

    def ipc_us(self, peer_export: bytes, nbytes: int, reps: int = 5) -> float:
        out = c_double()
        if self.lib.gs_probe_ipc(self.h, peer_export, int(nbytes), int(reps), byref(out)) != 0:
            raise RuntimeError(last_error(self.lib))
        return float(out.value)

    def rccl_init(self, uid: bytes, nranks: int, rank: int) -> None:
        if self.lib.gs_probe_rccl_init(self.h, uid, int(nranks), int(rank)) != 0:
            raise RuntimeError(last_error(self.lib))

    def rccl_us(self, peer: int, nbytes: int, reps: int = 5) -> float:
        out = c_double()
        if self.lib.gs_probe_rccl(self.h, int(peer), int(nbytes), int(reps), byref(out)) != 0:
            raise RuntimeError(last_error(self.lib))
        return float(out.value)

    def close(self) -> None:
        h, self.h = getattr(self, "h", None), None
        if h:
            self.lib.gs_probe_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # pragma: no cover - interpreter teardown
            pass
