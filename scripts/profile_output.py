#!/usr/bin/env python3
"""Host-side cost of one output step, broken down.

Runs a settings file end to end through the driver (default: the reference's example,
examples/settings-files.toml: L=64, 1000 steps, output every 10) with timing wrappers around
every host-side piece of the output path, and prints per-call means:

  sync            sim.synchronize() (the driver's phase timer waits for the device around phases)
  snapshot        GrayScott.snapshot_fields: compaction launch, D2H enqueue on the I/O stream
    native_call   the one C call that does it (HipBackend::snapshot)
  commit          SimulationOutput._commit_oldest: join the data write, gather, metadata
    join          the writer thread's job result (waits for its data write)
    gather        ctx.gather_object of the metadata blob
    metadata      BP4Writer.write_metadata (md.0 / md.idx appends, rank 0)
  writer thread   BP4Writer.put (block min / max + data write) and end_step, per call
  write_step      SimulationOutput.write_step as a whole (main thread)

  python scripts/profile_output.py [settings.toml] [--backend AMDGPU] [--out /tmp/gs_prof.bp]
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys
import tempfile
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STATS = collections.defaultdict(lambda: [0, 0.0])
_LOCK = threading.Lock()


def wrap(owner, name, label):
    fn = getattr(owner, name)

    def timed(*a, **k):
        t0 = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            dt = time.perf_counter() - t0
            with _LOCK:
                s = STATS[label]
                s[0] += 1
                s[1] += dt

    setattr(owner, name, timed)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("config", nargs="?", default=os.path.join(ROOT, "examples", "settings-files.toml"))
    ap.add_argument("--backend", default="AMDGPU")
    ap.add_argument("--out", default="")
    ap.add_argument("--repeat", type=int, default=2, help="runs (the first warms the page cache)")
    ap.add_argument("--torch-snapshot", action="store_true",
                    help="the snapshot through torch calls instead of the native one (A/B)")
    ap.add_argument("--queue", type=int, default=0, help="output_queue (0: the setting's)")
    ap.add_argument("--cprofile", action="store_true",
                    help="also print the main thread's cProfile of the last run (top 25 by own time)")
    a = ap.parse_args(argv)

    from grayscott_amd import driver
    from grayscott_amd.io import bp4, output
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.dist import DistContext
    from grayscott_amd.utils.config import get_settings

    GrayScott.native_snapshot = not a.torch_snapshot
    wrap(GrayScott, "synchronize", "sync")
    wrap(GrayScott, "snapshot_fields", "snapshot")
    from grayscott_amd.ops import native
    wrap(native.Engine, "snapshot", "snapshot.native_call")
    wrap(GrayScott, "_snapshot_views", "snapshot.views")
    wrap(output.SimulationOutput, "_commit_oldest", "commit")
    wrap(output.SimulationOutput, "write_step", "write_step")
    wrap(output._Job, "result", "commit.join")
    wrap(DistContext, "gather_object", "commit.gather")
    wrap(bp4.BP4Writer, "write_metadata", "commit.metadata")
    wrap(bp4.BP4Writer, "put", "writer.put")
    wrap(bp4.BP4Writer, "end_step", "writer.end_step")
    results = []
    for r in range(a.repeat):
        STATS.clear()
        s = get_settings([a.config])
        s.backend = a.backend
        if a.queue:
            s.output_queue = a.queue
        s.output = a.out or os.path.join(tempfile.gettempdir(), f"gs_prof_{os.getpid()}_{r}.bp")
        pr = None
        if a.cprofile and r == a.repeat - 1:
            import cProfile
            pr = cProfile.Profile()
            pr.enable()
        res = driver.run(s, out=open(os.devnull, "w"))
        if pr is not None:
            pr.disable()
            import pstats
            pstats.Stats(pr, stream=sys.stderr).sort_stats("tottime").print_stats(25)
        steps_out = STATS["write_step"][0]
        rec = {"run": r, "snapshot": "torch" if a.torch_snapshot else "native",
               "queue": s.output_queue, "loop_s": round(res["loop_s"], 5), "compute_s": round(res["compute_s"], 5),
               "output_s": round(res["timers"].get("output", {}).get("seconds", 0.0), 5),
               "output_steps": steps_out,
               "per_call_us": {k: round(1e6 * v[1] / max(1, v[0]), 1) for k, v in sorted(STATS.items())},
               "calls": {k: v[0] for k, v in sorted(STATS.items())}}
        results.append(rec)
        print(json.dumps(rec), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
