"""ADIOS2 BP4 files: native writer (libgs_core.so, csrc/io/bp4.cpp) + pure-Python reader.

Replaces ADIOS2.jl/libadios2 (reference src/simulation/IO.jl).  A ``<name>.bp`` directory holds
``data.<rank>`` subfiles (one process group per step per rank), ``md.0`` (per-step PG,
variable and attribute indices merged over ranks) and ``md.idx`` (64-byte record per step).
The byte layout is documented in docs/BP4_FORMAT.md.

The reader is an independent implementation (it shares no code with the C++ writer), so the
round-trip tests check the serialization from both ends.  It supports reading any box of a
global array from any step, regardless of the decomposition that wrote it -- which is what
restart-with-a-different-rank-count and the PDF analysis need.
"""
from __future__ import annotations

import ctypes
import os
import struct
from ctypes import POINTER, c_char_p, c_int32, c_int64, c_uint64, c_void_p
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..ops import native

# BP4 data-type ids (ADIOS2 BPBase::DataTypes)
TYPE_BYTE, TYPE_SHORT, TYPE_INTEGER, TYPE_LONG = 0, 1, 2, 4
TYPE_REAL, TYPE_DOUBLE, TYPE_STRING, TYPE_STRING_ARRAY = 5, 6, 9, 12
TYPE_UBYTE, TYPE_USHORT, TYPE_UINT, TYPE_ULONG = 50, 51, 52, 54

NP_TO_BP = {
    np.dtype(np.int8): TYPE_BYTE, np.dtype(np.int16): TYPE_SHORT,
    np.dtype(np.int32): TYPE_INTEGER, np.dtype(np.int64): TYPE_LONG,
    np.dtype(np.float32): TYPE_REAL, np.dtype(np.float64): TYPE_DOUBLE,
    np.dtype(np.uint8): TYPE_UBYTE, np.dtype(np.uint16): TYPE_USHORT,
    np.dtype(np.uint32): TYPE_UINT, np.dtype(np.uint64): TYPE_ULONG,
}
BP_TO_NP = {v: k for k, v in NP_TO_BP.items()}

CH_VALUE, CH_MIN, CH_MAX, CH_OFFSET, CH_DIMS = 0, 1, 2, 3, 4
CH_VAR_ID, CH_PAYLOAD_OFFSET, CH_FILE_INDEX, CH_TIME_INDEX = 5, 6, 7, 8
CH_BITMAP, CH_STAT, CH_TRANSFORM, CH_MINMAX = 9, 10, 11, 12


class BP4Error(RuntimeError):
    pass


# ------------------------------------------------------------------------------------------
# writer (native)
# ------------------------------------------------------------------------------------------
def _lib():
    lib = native.load("core")
    if not getattr(lib, "_bp4_declared", False):
        lib.bp4_open.restype = c_void_p
        lib.bp4_open.argtypes = [c_char_p, c_char_p, c_int32, c_int32, c_int32]
        lib.bp4_open_append.restype = c_void_p
        lib.bp4_open_append.argtypes = [c_char_p, c_char_p, c_int32, c_int32, c_int32,
                                        ctypes.c_uint32, c_int64, c_int64, c_int64]
        lib.bp4_last_error.restype = c_char_p
        lib.bp4_define_attribute.argtypes = [c_void_p, c_char_p, c_int32, c_void_p, c_int64]
        lib.bp4_define_attribute.restype = c_int32
        lib.bp4_define_variable.argtypes = [c_void_p, c_char_p, c_int32, c_int32,
                                            POINTER(c_uint64), POINTER(c_uint64),
                                            POINTER(c_uint64)]
        lib.bp4_define_variable.restype = c_int32
        lib.bp4_set_selection.argtypes = [c_void_p, c_int32, POINTER(c_uint64), POINTER(c_uint64)]
        lib.bp4_begin_step.argtypes = [c_void_p]
        lib.bp4_begin_step.restype = c_int32
        lib.bp4_put.argtypes = [c_void_p, c_int32, c_void_p]
        lib.bp4_put.restype = c_int32
        lib.bp4_put_minmax.argtypes = [c_void_p, c_int32, c_void_p, ctypes.c_double, ctypes.c_double]
        lib.bp4_put_minmax.restype = c_int32
        lib.bp4_write_step_uv.argtypes = [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32,
                                          c_void_p, c_void_p, c_int32]
        lib.bp4_write_step_uv.restype = c_int32
        lib.bp4_async_submit.argtypes = [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                                         c_void_p, c_int32, c_void_p, c_void_p, c_int32]
        lib.bp4_async_submit.restype = c_int64
        lib.bp4_async_result.argtypes = [c_void_p, c_int64, POINTER(ctypes.POINTER(ctypes.c_char)),
                                         POINTER(c_int64)]
        lib.bp4_async_result.restype = c_int32
        lib.bp4_end_step.argtypes = [c_void_p]
        lib.bp4_end_step.restype = c_int32
        lib.bp4_step_metadata.argtypes = [c_void_p, POINTER(ctypes.POINTER(ctypes.c_char))]
        lib.bp4_step_metadata.restype = c_int64
        lib.bp4_write_metadata.argtypes = [c_void_p, c_int32, POINTER(c_char_p), POINTER(c_int64)]
        lib.bp4_write_metadata.restype = c_int32
        lib.bp4_close.argtypes = [c_void_p]
        lib.bp4_close.restype = c_int32
        lib.bp4_flush.argtypes = [c_void_p]
        lib.bp4_flush.restype = c_int32
        lib._bp4_declared = True
    return lib


def _u64s(vals):
    vals = [int(v) for v in vals]
    return (c_uint64 * max(1, len(vals)))(*vals)


class BP4Writer:
    """One rank's handle on a BP4 output.  Rank 0 also owns md.0 / md.idx."""

    def __init__(self, path: str, io_name: str, rank: int = 0, nranks: int = 1,
                 column_major: bool = False, append: Optional[Dict[str, Any]] = None):
        """``append``: continue an existing file after its first ``append["steps"]`` steps (an
        :func:`append_plan`, the same on every rank; later steps are cut off)."""
        self.lib = _lib()
        self.path, self.rank, self.nranks = path, rank, nranks
        if append:
            h = self.lib.bp4_open_append(path.encode(), io_name.encode(), rank, nranks,
                                         1 if column_major else 0, int(append["steps"]),
                                         int(append["data_end"].get(rank, -1)),
                                         int(append["md_end"]), int(append["idx_end"]))
        else:
            h = self.lib.bp4_open(path.encode(), io_name.encode(), rank, nranks,
                                  1 if column_major else 0)
        if not h:
            raise BP4Error(self.lib.bp4_last_error().decode())
        self.h = c_void_p(h)
        self._vars: Dict[str, Tuple[int, np.dtype, Tuple[int, ...]]] = {}

    def _chk(self, rc, what):
        if rc != 0:
            raise BP4Error(f"{what}: {self.lib.bp4_last_error().decode()}")

    def define_attribute(self, name: str, value: Any) -> None:
        if isinstance(value, str):
            arr = (c_char_p * 1)(value.encode())
            self._chk(self.lib.bp4_define_attribute(self.h, name.encode(), TYPE_STRING, arr, 1), name)
            return
        if isinstance(value, (list, tuple)) and value and all(isinstance(v, str) for v in value):
            arr = (c_char_p * len(value))(*[v.encode() for v in value])
            self._chk(self.lib.bp4_define_attribute(self.h, name.encode(), TYPE_STRING_ARRAY, arr,
                                                    len(value)), name)
            return
        a = np.ascontiguousarray(np.atleast_1d(np.asarray(value)))
        if a.dtype == np.bool_:
            a = a.astype(np.uint8)
        if a.dtype.kind == "f":
            a = a.astype(np.float64) if a.dtype != np.float32 else a
        if a.dtype.kind in "iu" and a.dtype not in NP_TO_BP:
            a = a.astype(np.int64)
        self._chk(self.lib.bp4_define_attribute(self.h, name.encode(), NP_TO_BP[a.dtype],
                                                a.ctypes.data, a.size), name)

    def define_variable(self, name: str, dtype, shape: Sequence[int] = (),
                        start: Sequence[int] = (), count: Sequence[int] = ()) -> int:
        dt = np.dtype(dtype)
        vid = self.lib.bp4_define_variable(self.h, name.encode(), NP_TO_BP[dt], len(count),
                                           _u64s(shape), _u64s(start), _u64s(count))
        if vid < 0:
            raise BP4Error(self.lib.bp4_last_error().decode())
        self._vars[name] = (vid, dt, tuple(int(c) for c in count))
        return vid

    def set_selection(self, name: str, start: Sequence[int], count: Sequence[int]) -> None:
        vid, dt, _ = self._vars[name]
        self.lib.bp4_set_selection(self.h, vid, _u64s(start), _u64s(count))
        self._vars[name] = (vid, dt, tuple(int(c) for c in count))

    def begin_step(self) -> None:
        self._chk(self.lib.bp4_begin_step(self.h), "begin_step")

    def put(self, name: str, data, minmax=None) -> None:
        """Append this rank's block of ``name``.  ``minmax``: the block's (min, max), when the
        caller already has them (the GPU snapshot computes them, GrayScott.snapshot_fields), so
        the writer does not scan the block for its characteristics."""
        vid, dt, count = self._vars[name]
        a = np.ascontiguousarray(np.asarray(data, dtype=dt))
        if count and a.shape != count:
            raise BP4Error(f"{name}: block shape {a.shape} != count {count}")
        if not count and a.size != 1:
            raise BP4Error(f"{name}: single value expected")
        if minmax is not None and count:
            self._chk(self.lib.bp4_put_minmax(self.h, vid, a.ctypes.data, float(minmax[0]),
                                              float(minmax[1])), f"put {name}")
        else:
            self._chk(self.lib.bp4_put(self.h, vid, a.ctypes.data), f"put {name}")

    def write_step_uv(self, step: int, u, v, part=None) -> bytes:
        """One whole step -- begin, ``step``, ``U``, ``V`` (min / max reduced from the snapshot
        kernel's per-chunk quadruples ``part``, or scanned when None), end -- in one native call
        (the GIL is released for the entire data write); returns the metadata blob."""
        _, dt, count = self._vars["U"]
        for a in (u, v):
            if a.dtype != dt or a.shape != count or not a.flags.c_contiguous:
                raise BP4Error(f"write_step_uv: blocks must be C-contiguous {np.dtype(dt).name} {count}")
        st = np.int32(step)
        pp = part.ctypes.data if part is not None and len(part) else None
        self._chk(self.lib.bp4_write_step_uv(
            self.h, self._vars["step"][0], int(st), self._vars["U"][0], u.ctypes.data,
            self._vars["V"][0], v.ctypes.data, pp, len(part) if pp else 0), "write_step_uv")
        ptr = ctypes.POINTER(ctypes.c_char)()
        n = self.lib.bp4_step_metadata(self.h, ctypes.byref(ptr))
        return ctypes.string_at(ptr, n)

    def submit_step_uv(self, step: int, u, v, part=None, wait_fn=None, wait_arg=None) -> int:
        """Queue ``write_step_uv`` on the writer's native thread (started on first use), after
        ``wait_fn(wait_arg)`` -- a C function pointer, e.g. libgs_hip's ``gs_event_sync`` on the
        snapshot's copy event -- returns.  No Python runs on that thread.  ``u``, ``v``,
        ``part`` must stay alive until ``step_result`` returns for the ticket."""
        _, dt, count = self._vars["U"]
        for a in (u, v):
            if a.dtype != dt or a.shape != count or not a.flags.c_contiguous:
                raise BP4Error(f"submit_step_uv: blocks must be C-contiguous {np.dtype(dt).name} {count}")
        pp = part.ctypes.data if part is not None and len(part) else None
        t = self.lib.bp4_async_submit(self.h, wait_fn, wait_arg, self._vars["step"][0],
                                      int(np.int32(step)), self._vars["U"][0], u.ctypes.data,
                                      self._vars["V"][0], v.ctypes.data, pp,
                                      len(part) if pp else 0)
        if t < 0:
            raise BP4Error("submit_step_uv: " + self.lib.bp4_last_error().decode())
        return int(t)

    def step_result(self, ticket: int) -> bytes:
        """Wait for a queued step; its metadata blob (raises the step's error)."""
        ptr = ctypes.POINTER(ctypes.c_char)()
        n = c_int64(0)
        self._chk(self.lib.bp4_async_result(self.h, int(ticket), ctypes.byref(ptr), ctypes.byref(n)),
                  "async step")
        return ctypes.string_at(ptr, n.value)

    def end_step(self) -> bytes:
        """Close the step's process group; returns this rank's metadata blob."""
        self._chk(self.lib.bp4_end_step(self.h), "end_step")
        ptr = ctypes.POINTER(ctypes.c_char)()
        n = self.lib.bp4_step_metadata(self.h, ctypes.byref(ptr))
        return ctypes.string_at(ptr, n)

    def write_metadata(self, blobs: List[bytes]) -> None:
        arr = (c_char_p * len(blobs))(*blobs)
        sizes = (c_int64 * len(blobs))(*[len(b) for b in blobs])
        self._chk(self.lib.bp4_write_metadata(self.h, len(blobs), arr, sizes), "write_metadata")

    def flush(self) -> None:
        self.lib.bp4_flush(self.h)

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.bp4_close(self.h)
            self.h = None


def append_plan(path: str, keep_until_step: int, step_var: str = "step") -> Optional[Dict[str, Any]]:
    """How to continue the BP4 output at ``path`` after a restart at ``keep_until_step``: keep
    the leading steps whose ``step_var`` value is <= ``keep_until_step`` and cut off the rest.
    Returns ``{"steps", "last_step", "md_end", "idx_end", "data_end": {subfile: bytes}}`` or
    None when there is nothing to keep (no file, unreadable, or no step qualifies).  Read by
    one rank and broadcast; every rank then opens its subfile with ``BP4Writer(append=...)``."""
    try:
        rd = BP4Reader(path)
    except (BP4Error, OSError, struct.error):
        return None
    try:
        keep, last = 0, None
        for i in range(rd.steps):
            try:
                v = int(rd.read(step_var, i))
            except BP4Error:
                break
            if v > keep_until_step:
                break
            keep, last = i + 1, v
        if keep == 0:
            return None
        data_end: Dict[int, int] = {}
        for i in range(keep):
            for pg in rd.process_groups(i):
                k = int(pg["rank"])
                fh = rd._file(k)
                fh.seek(pg["offset"])
                (ln,) = struct.unpack("<Q", fh.read(8))
                data_end[k] = max(data_end.get(k, 0), int(pg["offset"]) + 8 + int(ln))
        return {"steps": keep, "last_step": last, "md_end": int(rd.records[keep - 1][5]),
                "idx_end": 64 + 64 * keep, "data_end": data_end, "shapes": {
                    n: tuple(vi.shape) for n, vi in rd.variables(keep - 1).items()},
                "dtypes": {n: str(vi.dtype) for n, vi in rd.variables(keep - 1).items()}}
    finally:
        rd.close()


# ------------------------------------------------------------------------------------------
# reader (pure Python)
# ------------------------------------------------------------------------------------------
class _Cur:
    def __init__(self, buf: bytes, pos: int = 0):
        self.b, self.p = buf, pos

    def take(self, fmt: str):
        v = struct.unpack_from("<" + fmt, self.b, self.p)
        self.p += struct.calcsize("<" + fmt)
        return v if len(v) > 1 else v[0]

    def raw(self, n: int) -> bytes:
        v = self.b[self.p:self.p + n]
        self.p += n
        return v

    def name(self) -> str:
        n = self.take("H")
        return self.raw(n).decode()


@dataclass
class Block:
    step: int
    file_index: int
    count: Tuple[int, ...]
    shape: Tuple[int, ...]
    start: Tuple[int, ...]
    payload_offset: int
    var_offset: int
    value: Any = None
    vmin: Any = None
    vmax: Any = None


@dataclass
class VarInfo:
    name: str
    type: int
    blocks: List[Block] = field(default_factory=list)

    @property
    def dtype(self) -> np.dtype:
        return BP_TO_NP[self.type]

    @property
    def shape(self) -> Tuple[int, ...]:
        return self.blocks[0].shape if self.blocks else ()

    @property
    def is_single_value(self) -> bool:
        return bool(self.blocks) and not self.blocks[0].count


def _type_size(t: int) -> int:
    return BP_TO_NP[t].itemsize


def _parse_charset(c: _Cur, vtype: int, is_attr: bool):
    n = c.take("B")
    length = c.take("I")
    end = c.p + length
    out: Dict[str, Any] = {}
    for _ in range(n):
        cid = c.take("B")
        if cid == CH_TIME_INDEX:
            out["step"] = c.take("I")
        elif cid == CH_FILE_INDEX:
            out["file_index"] = c.take("I")
        elif cid == CH_DIMS:
            nd = c.take("B")
            c.take("H")
            dims = [c.take("QQQ") for _ in range(nd)]
            out["count"] = tuple(d[0] for d in dims)
            out["shape"] = tuple(d[1] for d in dims)
            out["start"] = tuple(d[2] for d in dims)
        elif cid == CH_VALUE:
            if is_attr:
                if vtype == TYPE_STRING:
                    out["value"] = c.raw(c.take("H")).decode()
                elif vtype == TYPE_STRING_ARRAY:
                    k = c.take("I")
                    out["value"] = [c.raw(c.take("H")).decode() for _ in range(k)]
                else:
                    k = c.take("H")
                    arr = np.frombuffer(c.raw(k * _type_size(vtype)), dtype=BP_TO_NP[vtype])
                    out["value"] = arr[0].item() if k == 1 else arr.copy()
            else:
                ts = _type_size(vtype)
                out["value"] = np.frombuffer(c.raw(ts), dtype=BP_TO_NP[vtype])[0].item()
        elif cid == CH_MINMAX:
            m = c.take("H")
            ts = _type_size(vtype)
            mm = np.frombuffer(c.raw(2 * ts), dtype=BP_TO_NP[vtype])
            out["min"], out["max"] = mm[0].item(), mm[1].item()
            if m > 1:
                raise BP4Error("sub-block statistics are not supported")
        elif cid in (CH_MIN, CH_MAX):
            ts = _type_size(vtype)
            out["min" if cid == CH_MIN else "max"] = \
                np.frombuffer(c.raw(ts), dtype=BP_TO_NP[vtype])[0].item()
        elif cid == CH_OFFSET:
            out["offset"] = c.take("Q")
        elif cid == CH_PAYLOAD_OFFSET:
            out["payload_offset"] = c.take("Q")
        elif cid == CH_VAR_ID:
            out["var_id"] = c.take("I")
        else:  # unknown characteristic: skip the rest of the set
            break
    c.p = end
    return out


class BP4Reader:
    """Reads BP4 directories written by :class:`BP4Writer` (any number of writer ranks)."""

    def __init__(self, path: str):
        self.path = path
        idx_path = os.path.join(path, "md.idx")
        md_path = os.path.join(path, "md.0")
        if not (os.path.exists(idx_path) and os.path.exists(md_path)):
            raise BP4Error(f"{path} is not a BP4 directory")
        with open(idx_path, "rb") as fh:
            idx = fh.read()
        with open(md_path, "rb") as fh:
            self._md = fh.read()
        self.header = self._check_header(idx, b"I")
        self._check_header(self._md, b"M")
        self.active = idx[38] == 1
        self.records = []
        for off in range(64, len(idx) - 63, 64):
            rec = struct.unpack_from("<8Q", idx, off)
            self.records.append(rec)
        self.attributes: Dict[str, Any] = {}
        self._steps: List[Dict[str, VarInfo]] = []
        self._pgs: List[list] = []
        for rec in self.records:
            self._parse_step(rec)
        self._files: Dict[int, Any] = {}

    @staticmethod
    def _check_header(buf: bytes, kind: bytes) -> Dict[str, Any]:
        if len(buf) < 64 or not buf.startswith(b"ADIOS-BP v"):
            raise BP4Error("bad BP header")
        if buf[31:32] != kind:
            raise BP4Error(f"header kind {buf[31:32]!r} != {kind!r}")
        if buf[37] != 4:
            raise BP4Error(f"not a BP4 file (version byte {buf[37]})")
        if buf[36] != 0:
            raise BP4Error("big-endian BP files are not supported")
        return {"tag": buf[:32].decode().strip(), "minor": buf[39]}

    def _parse_step(self, rec) -> None:
        step, _, pg_start, vars_start, attrs_start, end, _, _ = rec
        c = _Cur(self._md, pg_start)
        npg = c.take("Q")
        c.take("Q")
        pgs = []
        for _ in range(npg):
            ln = c.take("H")
            e = c.p + ln
            io = c.name()
            colmaj = c.raw(1)
            prank = c.take("I")
            c.name()
            ts = c.take("I")
            off = c.take("Q")
            pgs.append({"io": io, "column_major": colmaj == b"y", "rank": prank, "step": ts,
                        "offset": off})
            c.p = e
        self._pgs.append(pgs)
        c = _Cur(self._md, vars_start)
        nvars = c.take("I")
        c.take("Q")
        variables: Dict[str, VarInfo] = {}
        for _ in range(nvars):
            ln = c.take("I")
            e = c.p + ln
            c.take("I")  # member id
            c.name()     # group
            vname = c.name()
            c.name()     # path
            vtype = c.take("B")
            nsets = c.take("Q")
            vi = VarInfo(vname, vtype)
            for _ in range(nsets):
                ch = _parse_charset(c, vtype, False)
                vi.blocks.append(Block(step=ch.get("step", step), file_index=ch.get("file_index", 0),
                                       count=ch.get("count", ()), shape=ch.get("shape", ()),
                                       start=ch.get("start", ()),
                                       payload_offset=ch.get("payload_offset", 0),
                                       var_offset=ch.get("offset", 0), value=ch.get("value"),
                                       vmin=ch.get("min"), vmax=ch.get("max")))
            variables[vname] = vi
            c.p = e
        self._steps.append(variables)
        c = _Cur(self._md, attrs_start)
        nattrs = c.take("I")
        c.take("Q")
        for _ in range(nattrs):
            ln = c.take("I")
            e = c.p + ln
            c.take("I")
            c.name()
            aname = c.name()
            c.name()
            atype = c.take("B")
            c.take("Q")
            ch = _parse_charset(c, atype, True)
            self.attributes[aname] = ch.get("value")
            c.p = e

    # ---------------------------------------------------------------------------------
    @property
    def steps(self) -> int:
        return len(self._steps)

    def variables(self, step: int = 0) -> Dict[str, VarInfo]:
        return self._steps[step]

    def process_groups(self, step: int = 0) -> list:
        return self._pgs[step]

    def _file(self, k: int):
        if k not in self._files:
            self._files[k] = open(os.path.join(self.path, f"data.{k}"), "rb")
        return self._files[k]

    def _block_data(self, b: Block, dtype: np.dtype) -> np.ndarray:
        n = int(np.prod(b.count)) if b.count else 1
        fh = self._file(b.file_index)
        fh.seek(b.payload_offset)
        raw = fh.read(n * dtype.itemsize)
        if len(raw) != n * dtype.itemsize:
            raise BP4Error("truncated data file")
        return np.frombuffer(raw, dtype=dtype).reshape(b.count if b.count else ())

    def _block_view(self, b: Block, dtype: np.dtype) -> np.ndarray:
        """Array block as a read-only memory map: a (sub-box) selection copies only the pages
        it touches, once (checkpoint restarts read 512 MB blocks)."""
        n = int(np.prod(b.count))
        fh = self._file(b.file_index)
        if os.fstat(fh.fileno()).st_size < b.payload_offset + n * dtype.itemsize:
            raise BP4Error("truncated data file")
        return np.memmap(fh, dtype=dtype, mode="r", offset=b.payload_offset, shape=tuple(b.count))

    def read(self, name: str, step: int = -1, start: Optional[Sequence[int]] = None,
             count: Optional[Sequence[int]] = None):
        """Read a variable at ``step`` (negative = from the end), optionally a sub-box."""
        if step < 0:
            step += self.steps
        if not 0 <= step < self.steps:
            raise BP4Error(f"step {step} out of range (0..{self.steps - 1})")
        vi = self._steps[step].get(name)
        if vi is None:
            raise BP4Error(f"variable {name!r} not in step {step}")
        dt = vi.dtype
        if vi.is_single_value:
            b = vi.blocks[0]
            return b.value if b.value is not None else self._block_data(b, dt).item()
        shape = vi.shape
        start = tuple(start) if start is not None else (0,) * len(shape)
        count = tuple(count) if count is not None else tuple(s - o for s, o in zip(shape, start))
        out = np.empty(count, dtype=dt)
        filled = 0
        for b in vi.blocks:
            lo = [max(s, bs) for s, bs in zip(start, b.start)]
            hi = [min(s + c, bs + bc) for s, c, bs, bc in zip(start, count, b.start, b.count)]
            if any(h <= l for l, h in zip(lo, hi)):
                continue
            data = self._block_view(b, dt)
            src = tuple(slice(l - bs, h - bs) for l, h, bs in zip(lo, hi, b.start))
            dst = tuple(slice(l - s, h - s) for l, h, s in zip(lo, hi, start))
            out[dst] = data[src]
            filled += int(np.prod([h - l for l, h in zip(lo, hi)]))
        if filled != int(np.prod(count)):
            raise BP4Error(f"{name}: selection not fully covered by written blocks")
        return out

    def close(self) -> None:
        for fh in self._files.values():
            fh.close()
        self._files.clear()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
