"""Simulation output stream (reference src/simulation/IO.jl).

Parity:
  * ``init``          -- IO.jl:37-70: IO "SimulationOutput", provenance attributes F, k, dt, Du,
                         Dv, noise (Float64), Fides + VTX visualization schemas (IO.jl:123-163),
                         variables ``step`` (Int32 global value), ``U``/``V`` (global L^3 arrays,
                         per-rank blocks)
  * ``write_step``    -- IO.jl:82-96: ghost-free copy (get_fields), begin_step, put step/U/V,
                         end_step
  * ``close``         -- IO.jl:107-110

Arrays are declared row-major like the ADIOS2 C++ gray-scott example: shape {Lz,Ly,Lx},
start {oz,oy,ox}, count {nz,ny,nx} with x fastest in memory -- the same bytes as the Julia
column-major (x,y,z) declaration.  Each rank writes its own ``data.<rank>`` subfile; rank 0
gathers the per-rank step metadata over the control plane and writes md.0 / md.idx.  The
GPU->host copy uses the compaction kernel (no full-buffer D2H as in the reference, D1/K14).

``async_output`` (default true): a step is written behind the simulation -- device snapshot and
D2H on an I/O stream, the data write on a host thread.  Up to ``output_queue`` (default 2) steps
are in flight: ``write_step`` first commits the oldest ones (joins its data write, gathers and
writes its metadata) until fewer are pending, so step n is complete in the file once step
n + output_queue starts (or the stream is closed), and the main thread's own per-step work
(metadata gather, the next snapshot) overlaps the previous step's data write instead of
following it.  Snapshots above 1 GiB per rank keep one step in flight (the pinned host
buffers are per queued step; such steps are write-bound).  ``async_output = false`` writes
each step before ``write_step`` returns.

Restart (``append_after_step``): the output history is kept -- the existing file's steps up to
the restart step stay, later ones (written after the checkpoint by the failed run) are cut off,
and the run appends from there (the ADIOS2 append semantics the reference's restart hook,
GrayScott.jl:77-78, implies).
"""
from __future__ import annotations

import collections
import os
import shutil
from typing import Optional

import numpy as np

from ..parallel.dist import DistContext
from .bp4 import BP4Writer

_NP = {"float32": np.float32, "float64": np.float64}
# pinned (page-locked) host memory the asynchronous output ring may hold per rank: the queue
# depth is cut to what fits (a 512^3 fp32 rank's 1 GiB snapshot: one step in flight)
PINNED_RING_BYTES = 1 << 30


def vtk_schema(L) -> str:
    """VTX ImageData schema (IO.jl:137-157): extents "0 L 0 L 0 L", cell data U, V, TIME."""
    if isinstance(L, int):
        L = (L, L, L)
    extent = " ".join(f"0 {int(v)}" for v in L)
    return (
        '\n        <?xml version="1.0"?>\n'
        '        <VTKFile type="ImageData" version="0.1" byte_order="LittleEndian">\n'
        f'          <ImageData WholeExtent="{extent}" Origin="0 0 0" Spacing="1 1 1">\n'
        f'            <Piece Extent="{extent}">\n'
        '              <CellData Scalars="U">\n'
        '                <DataArray Name="U" />\n'
        '                <DataArray Name="V" />\n'
        '                <DataArray Name="TIME">\n'
        '                  step\n'
        '                </DataArray>\n'
        '              </CellData>\n'
        '            </Piece>\n'
        '          </ImageData>\n'
        '        </VTKFile>')


def add_visualization_schemas(w: BP4Writer, L) -> None:
    """Fides + VTX attributes (IO.jl:123-163)."""
    w.define_attribute("Fides_Data_Model", "uniform")
    w.define_attribute("Fides_Origin", [0.0, 0.0, 0.0])
    w.define_attribute("Fides_Spacing", [0.1, 0.1, 0.1])
    w.define_attribute("Fides_Dimension_Variable", "U")
    w.define_attribute("Fides_Variable_List", ["U", "V"])
    w.define_attribute("Fides_Variable_Associations", ["points", "points"])
    w.define_attribute("vtk.xml", vtk_schema(L))


def _prepare_dir(path: str, ctx: DistContext) -> None:
    if ctx.rank == 0 and os.path.isdir(path):
        shutil.rmtree(path)
    ctx.barrier()


def _append_plan(path: str, step: int, domain, dtype, ctx: DistContext):
    """Rank 0 decides whether (and where) the existing output at ``path`` is continued; the
    plan is broadcast so every rank opens its subfile consistently."""
    plan = None
    if ctx.rank == 0 and os.path.isdir(path):
        from .bp4 import append_plan
        plan = append_plan(path, step)
        Lx, Ly, Lz = domain.L
        if plan is not None and (plan["shapes"].get("U") != (Lz, Ly, Lx) or
                                 plan["dtypes"].get("U") != np.dtype(dtype).name):
            import warnings
            warnings.warn(f"{path}: existing output has another grid or precision; "
                          "starting a new file")
            plan = None
    return ctx.broadcast_object(plan, src=0)


class SimulationOutput:
    """ADIOSStream equivalent (IO.jl:15-22)."""

    IO_NAME = "SimulationOutput"

    def __init__(self, settings, domain, ctx: Optional[DistContext] = None, path: Optional[str] = None,
                 io_name: Optional[str] = None, schemas: bool = True,
                 append_after_step: Optional[int] = None):
        self.ctx = ctx or DistContext()
        self.settings = settings
        self.domain = domain
        self.path = path or settings.output
        dtype = _NP[settings.dtype_name]
        plan = None
        if append_after_step is not None:
            plan = _append_plan(self.path, int(append_after_step), domain, dtype, self.ctx)
        if plan is None:
            _prepare_dir(self.path, self.ctx)
        self.kept_steps = plan["steps"] if plan else 0
        self.last_step = plan["last_step"] if plan else None
        self.w = BP4Writer(self.path, io_name or self.IO_NAME, self.ctx.rank, self.ctx.world_size,
                           append=plan)
        if self.ctx.rank == 0:
            for key in ("F", "k", "dt", "Du", "Dv", "noise"):
                self.w.define_attribute(key, float(getattr(settings, key)))
            if schemas:
                add_visualization_schemas(self.w, domain.L)
        Lx, Ly, Lz = domain.L
        ox, oy, oz = domain.proc_offsets
        nx, ny, nz = domain.proc_sizes
        self.w.define_variable("step", np.int32)
        self.w.define_variable("U", dtype, (Lz, Ly, Lx), (oz, oy, ox), (nz, ny, nx))
        self.w.define_variable("V", dtype, (Lz, Ly, Lx), (oz, oy, ox), (nz, ny, nx))
        self.steps_written = 0
        self.async_io = bool(getattr(settings, "async_output", True))
        self.queue = min(4, max(1, int(getattr(settings, "output_queue", 2))))  # 1..4
        self._pending = collections.deque()  # data-write jobs of uncommitted steps, in order

    def define_attribute(self, name, value) -> None:
        if self.ctx.rank == 0:
            self.w.define_attribute(name, value)

    def write_fields(self, step: int, u: np.ndarray, v: np.ndarray) -> None:
        self.w.begin_step()
        self.w.put("step", np.int32(step))
        self.w.put("U", u)
        self.w.put("V", v)
        blob = self.w.end_step()
        blobs = self.ctx.gather_object(blob, dst=0)
        if self.ctx.rank == 0:
            self.w.write_metadata(blobs)
        self.steps_written += 1

    def write_step(self, step: int, sim):
        """IO.jl:82-96.  With ``async_output`` (default) the step is written behind the
        simulation: device snapshot + D2H on an I/O stream, data write on a host thread; the
        collective metadata gather of step n happens on the main thread when step
        n + queue is written (or at close), in step order, so no collective ever runs off the
        main thread.  Returns the snapshot ``(u, v, wait, mm)`` it writes from (None when
        synchronous), so an asynchronous checkpoint of the same step can share it; the caller
        must have finished every other reader of that snapshot before the output step that
        reuses its buffers (``queue`` steps later)."""
        if not self.async_io:
            u, v = sim.get_fields()
            self.write_fields(step, u, v)
            self.last_step = step
            return None
        # the ring of pinned host snapshots is bounded in bytes, not in steps: at most
        # PINNED_RING_BYTES per rank (queue x snapshot), so an 8-rank node pins <= 8 GiB for
        # output whatever the sub-domain size (one step in flight beyond that)
        depth = self._depth(sim)
        while len(self._pending) >= depth:
            self._commit_oldest()
        u, v, wait, mm = sim.snapshot_fields("output", depth=depth, minmax=True)
        snap = (u, v, wait, mm)
        part = getattr(mm, "part", None)
        fn, arg = _native_wait(wait)
        if fn is not None:
            # the whole step on the writer's native thread (bp4_async_submit): it waits for the
            # D2H copy itself (gs_event_sync) and writes; no Python runs beside the stepping
            t = self.w.submit_step_uv(step, u, v, part, fn, arg)
            self._pending.append((step, _Ticket(self.w, t, (u, v, part, wait))))
            self.last_step = step
            return snap

        def job():
            # two native calls, the GIL released throughout (a Python put sequence here held it
            # between calls and stalled the stepping thread's own native calls): the D2H wait,
            # then the whole step -- the snapshot kernel's min / max partials reduced in C++
            wait()
            return self.w.write_step_uv(step, u, v, getattr(mm, "part", None))

        self._pending.append((step, worker("gs-async-output").submit(job)))
        self.last_step = step
        return snap

    def _depth(self, sim) -> int:
        # the ring of pinned host snapshots is bounded in bytes, not in steps
        return max(1, min(self.queue, PINNED_RING_BYTES // max(1, _snapshot_bytes(sim))))

    def prepare(self, sim) -> None:
        """Before the time loop (the driver's io_init phase): allocate the asynchronous output's
        pinned host ring and events and take one snapshot into every ring slot, so the first
        output steps do not pay the pinned allocations, the copy engines' first use of each
        buffer or the snapshot kernel's code-object load inside the loop."""
        if self.async_io and hasattr(sim, "prepare_snapshots"):
            sim.prepare_snapshots("output", depth=self._depth(sim), minmax=True)

    def _commit_oldest(self) -> None:
        """Finish the oldest in-flight step: wait for its data write, gather the per-rank
        metadata blobs and let rank 0 append them to the index (rank 0's metadata writes touch
        md.0 / md.idx only, so they may run while a later step's data write is in flight)."""
        _, job = self._pending.popleft()
        blob = job.result()
        blobs = self.ctx.gather_object(blob, dst=0)
        if self.ctx.rank == 0:
            self.w.write_metadata(blobs)
        self.steps_written += 1

    def flush(self) -> None:
        """Commit every in-flight asynchronous step."""
        while self._pending:
            self._commit_oldest()

    def commit_through(self, step: int) -> None:
        """Commit the in-flight steps up to ``step``.  The driver calls it with the step before
        a checkpoint's: once that checkpoint is committed, every earlier output step is in the
        file, so a restart from it only has to rewrite the checkpoint step itself."""
        while self._pending and self._pending[0][0] <= step:
            self._commit_oldest()

    def close(self) -> None:
        self.flush()
        self.w.close()
        self.ctx.barrier()


def _native_wait(wait):
    """(C function pointer, argument) that waits like ``wait`` -- a snapshot's native event
    (libgs_hip gs_event_sync) or nothing to wait for (the CPU backend's ready arrays) -- or
    (None, None) when only the Python callable can (the torch-event snapshot A/B path)."""
    ev = getattr(wait, "__self__", None)
    if ev is None:  # the CPU backend's lambda: the arrays are ready
        return 0, None
    from ..ops import native
    if isinstance(ev, native.NativeEvent):
        import ctypes
        return ctypes.cast(ev.lib.gs_event_sync, ctypes.c_void_p).value, ev.ptr
    return None, None


class _Ticket:
    """A step queued on the BP4 writer's native thread; ``keep`` holds the arrays (and the
    event) it reads until its result is taken."""

    def __init__(self, w: BP4Writer, ticket: int, keep):
        self.w, self.ticket, self.keep = w, ticket, keep

    def result(self) -> bytes:
        try:
            return self.w.step_result(self.ticket)
        finally:
            self.keep = None


def _snapshot_bytes(sim) -> int:
    """Bytes of one rank's ghost-free (u, v) snapshot."""
    n = 1
    for d in sim.local_shape:
        n *= int(d)
    return 2 * n * np.dtype(_NP.get(str(getattr(sim, "dtype", "float32")), np.float32)).itemsize


class _Worker:
    """One persistent host thread running submitted functions in order.  A thread started per
    output step cost ~0.7 ms of the stepping loop's time (Thread.start waits for the new thread
    to be scheduled next to the busy stepping threads); one long-lived thread per stream does
    not.  ctypes releases the GIL during the BP4 writes."""

    def __init__(self, name: str):
        import queue
        import threading
        self._q = queue.SimpleQueue()
        self._t = threading.Thread(target=self._loop, name=name, daemon=True)
        self._t.start()

    def _loop(self):
        while True:
            job = self._q.get()
            if job is None:
                return
            job._run()

    def submit(self, fn) -> "_Job":
        job = _Job(fn, start=False)
        self._q.put(job)
        return job

    def close(self) -> None:
        self._q.put(None)
        self._t.join()


_WORKERS = {}


def worker(name: str) -> _Worker:
    """The process-wide worker thread ``name`` (created on first use)."""
    w = _WORKERS.get(name)
    if w is None:
        w = _WORKERS[name] = _Worker(name)
    return w


class _Job:
    """A function running on a host thread: its own (start=True) or a _Worker's."""

    def __init__(self, fn, start: bool = True):
        import threading
        self._fn = fn
        self._out = None
        self._err = None
        self._done = threading.Event()
        if start:
            threading.Thread(target=self._run, name="gs-async-job", daemon=True).start()

    def _run(self):
        try:
            self._out = self._fn()
        except BaseException as ex:  # re-raised on the main thread
            self._err = ex
        finally:
            self._done.set()

    def result(self):
        self._done.wait()
        if self._err is not None:
            raise self._err
        return self._out
