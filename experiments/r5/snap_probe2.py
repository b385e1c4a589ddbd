"""Where the output step's snapshot_fields host time goes in the example's loop cadence
(iterate 10 steps, snapshot, repeat): per-line timers around an instrumented copy.

  python experiments/r5/snap_probe2.py
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch  # noqa: F401
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    s = Settings(L=64, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1, noise=0.1,
                 backend="AMDGPU")
    sim = GrayScott(s, init_domain(64, 1, 0), fuse=3)
    sim.init_fields()
    acc = {}

    def tick(name, t0):
        t1 = time.perf_counter()
        acc[name] = acc.get(name, 0.0) + (t1 - t0)
        return t1

    n = 100
    for it in range(n + 5):
        if it == 5:
            acc.clear()
        t = time.perf_counter()
        sim.iterate(10)
        t = tick("iterate(10)", t)
        u, v, wait, mm = sim.snapshot_fields("output", depth=2, minmax=True)
        t = tick("snapshot_fields", t)
        wait()
        t = tick("wait", t)
    print(json.dumps({k: round(1e6 * v / n, 1) for k, v in acc.items()}), flush=True)
    # the same cadence with the output stream's native writer thread writing each snapshot
    import tempfile
    from grayscott_amd.io.output import SimulationOutput
    out = SimulationOutput(s, sim.domain, path=os.path.join(tempfile.gettempdir(), f"snap2_{os.getpid()}.bp"))
    for label in ("with writer", "with writer (again)"):
        acc.clear()
        for it in range(n):
            t = time.perf_counter()
            sim.iterate(10)
            t = tick("iterate(10)", t)
            out.write_step(it, sim)
            t = tick("write_step", t)
        out.flush()
        print(json.dumps({"what": label, **{k: round(1e6 * v / n, 1) for k, v in acc.items()}}), flush=True)
    import grayscott_amd.models.grayscott as gm
    orig = gm.GrayScott.snapshot_fields
    sn = {"t": 0.0}

    def timed(self, *a, **k):
        t0 = time.perf_counter()
        try:
            return orig(self, *a, **k)
        finally:
            sn["t"] += time.perf_counter() - t0
    gm.GrayScott.snapshot_fields = timed
    acc.clear()
    for it in range(n):
        sim.iterate(10)
        out.write_step(it, sim)
    out.flush()
    print(json.dumps({"what": "snapshot_fields inside write_step, with writer", "us": round(1e6 * sn["t"] / n, 1)}), flush=True)
    gm.GrayScott.snapshot_fields = orig
    out.close()
    # the same with the profiler on the snapshot
    import cProfile
    import pstats
    pr = cProfile.Profile()
    for it in range(50):
        sim.iterate(10)
        pr.enable()
        u, v, wait, mm = sim.snapshot_fields("output", depth=2, minmax=True)
        pr.disable()
        wait()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(12)
    sim.close()


if __name__ == "__main__":
    main()
