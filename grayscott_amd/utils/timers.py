"""Phase timers and the JSON-lines perf log.

The reference only wraps the whole run in ``@time`` (gray-scott.jl:12).  Here:

* ``DeviceTimer`` times the compute intervals of the time loop in stream order on the device
  (a pair of timing events on the compute stream, into which the engine joins its
  communication stream at the end of every pass) without synchronising anything: an interval is
  read once its end event has completed.  The per-phase split of a pass (pack, transport,
  unpack, inner, shell, ...) is the engine's own profiling window
  (``GrayScott.phase_profile``, csrc/include/gs/phase.h).
* ``PhaseTimer`` times host-side phases (output, checkpoint, restart) with the host clock
  around device-synchronised sections.
* ``PerfLog`` appends one JSON record per output interval when ``perf_log`` is set:
  ``{"step", "steps", "compute_s", "io_s", "mlups", ...}``.
"""
from __future__ import annotations

import json
import time
from collections import defaultdict
from contextlib import contextmanager
from typing import Callable, Dict, Optional


class PhaseTimer:
    def __init__(self, sync: Optional[Callable[[], None]] = None):
        self.sync = sync or (lambda: None)
        self.total: Dict[str, float] = defaultdict(float)
        self.calls: Dict[str, int] = defaultdict(int)

    @contextmanager
    def phase(self, name: str, sync: bool = True):
        """Time a host phase.  ``sync``: wait for the device on both sides, so queued device work
        is not counted in the phase (and the phase's own device work is); an asynchronous phase
        (the output step: stream-ordered snapshot, host-thread write) passes False and is timed on
        the host only -- a device wait there would stall the host's run-ahead every output step."""
        if sync:
            self.sync()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if sync:
                self.sync()
            self.total[name] += time.perf_counter() - t0
            self.calls[name] += 1

    def summary(self) -> Dict[str, Dict[str, float]]:
        return {k: {"seconds": v, "calls": self.calls[k]} for k, v in self.total.items()}


class DeviceTimer:
    """Stream-ordered interval timer.  ``device``: a torch CUDA (HIP) device whose current
    stream carries the work, or None for a synchronous (CPU) backend, timed by the host clock.

        tok = t.start(); ...enqueue work...; t.stop(tok, {"step": 10})
        for seconds, meta in t.completed(): ...      # intervals whose work has finished
        for seconds, meta in t.completed(wait=True): ...  # all of them (synchronises)
    """

    def __init__(self, device=None):
        self.device = device
        self.pending = []
        self.total = 0.0
        self.count = 0

    def start(self):
        if self.device is None:
            return time.perf_counter()
        import torch
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        return ev

    def stop(self, token, meta: dict) -> None:
        """End the interval begun by ``token``; ``meta`` (kept by reference, so it may still be
        filled in) is returned with the interval's seconds by ``completed``."""
        if self.device is None:
            self.pending.append((time.perf_counter() - token, None, meta))
            return
        import torch
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.device))
        self.pending.append((token, ev, meta))

    def completed(self, wait: bool = False):
        out, keep = [], []
        for a, b, meta in self.pending:
            if b is None:
                out.append((a, meta))
            elif wait or b.query():
                b.synchronize()
                out.append((a.elapsed_time(b) * 1e-3, meta))
            else:
                keep.append((a, b, meta))
        self.pending = keep
        for sec, _ in out:
            self.total += sec
            self.count += 1
        return out


class PerfLog:
    def __init__(self, path: str = "", enabled: bool = True):
        self.fh = open(path, "a", encoding="utf-8") if (path and enabled) else None

    def write(self, **rec) -> None:
        if self.fh:
            self.fh.write(json.dumps(rec) + "\n")
            self.fh.flush()

    def close(self) -> None:
        if self.fh:
            self.fh.close()
            self.fh = None
