#!/usr/bin/env python3
"""Stream-time cost of an event record between back-to-back fused passes (one GPU, one rank):
N T=3 passes issued as one advance, then one advance per pass with (a) nothing, (b) a
no-timing event (the engine's cross-stream marks), (c) a timing event (the phase window's
stamps), (d) a no-timing event plus a wait on it from a second stream, recorded in between.
Time per pass from events around the whole run; interleaved rounds.

  python scripts/event_cost.py --L 256 --passes 40 --rounds 5
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from grayscott_amd.models.grayscott import GrayScott  # noqa: E402
from grayscott_amd.parallel.decomp import init_domain  # noqa: E402
from grayscott_amd.utils.config import Settings  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=256)
    ap.add_argument("--passes", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    s = Settings(L=a.L, precision="Float32", noise=0.1, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                 backend="AMDGPU")
    sim = GrayScott(s, init_domain(a.L, 1, 0), fuse=3)
    sim.init_fields()
    sim.randomize_fields(seed=1)
    cur = torch.cuda.current_stream()
    side = torch.cuda.Stream()
    k = sim.depth
    sim.iterate(10 * k)
    torch.cuda.synchronize()

    def run(mode):
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record(cur)
        if mode == "one_call":
            sim.iterate(a.passes * k)
        else:
            for _ in range(a.passes):
                sim.iterate(k)
                if mode == "event":
                    torch.cuda.Event().record(cur)
                elif mode == "timing_event":
                    torch.cuda.Event(enable_timing=True).record(cur)
                elif mode == "event_wait":
                    e = torch.cuda.Event()
                    e.record(cur)
                    side.wait_event(e)
        t1.record(cur)
        t1.synchronize()
        return 1e3 * t0.elapsed_time(t1) / a.passes

    modes = ("one_call", "per_pass", "event", "timing_event", "event_wait")
    res = {m: [] for m in modes}
    for _ in range(a.rounds):
        for m in modes:
            res[m].append(run(m))
    for m in modes:
        v = sorted(res[m])
        print(f"L={a.L} {m:13s} us/pass median {v[len(v) // 2]:8.1f}  min {v[0]:8.1f}", flush=True)
    sim.close()


if __name__ == "__main__":
    main()
