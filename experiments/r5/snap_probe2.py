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
