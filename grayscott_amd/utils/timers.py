"""Phase timers and the JSON-lines perf log.

The reference only wraps the whole run in ``@time`` (gray-scott.jl:12).  Here every phase of
the driver is timed (host wall clock around device-synchronised sections) and, when
``perf_log`` is set, one JSON record per output interval is appended:
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
    def phase(self, name: str):
        self.sync()
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.sync()
            self.total[name] += time.perf_counter() - t0
            self.calls[name] += 1

    def summary(self) -> Dict[str, Dict[str, float]]:
        return {k: {"seconds": v, "calls": self.calls[k]} for k, v in self.total.items()}


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
