#!/usr/bin/env python3
"""Cost of a gated pass (csrc/hip/gate.hpp) against the full pass, on ONE MI355X.

One rank whose halo messages go to ITSELF through the IPC landing buffer (loopback, engine.h
set_loopback) on a non-periodic geometry: every exchange runs the real in-kernel protocol --
packers, counter, flags, bounded waits, cone unpacks -- with the sub-domain one rank of an
N-GPU job owns.  Per k-step pass (ms), for the neighbour sets:
  z      -- neighbours at -z / +z only (z slabs: whole-plane messages),
  all    -- all 26 directions (every face, edge and corner; the interior rank of a large grid);
  plus   -- +x, +y, +z faces, their edges and corner: a 2x2x2 rank of BASELINE config 3 (debug
            knob ipc_pair_same_dir: each message lands in its own direction's ghost box --
            timing only, the values are no wrap);
and the pass kinds:
  full       -- the fused pass of a rank without neighbours (no exchange): the floor,
  gated      -- the gated pass (the default for IPC, overlap on; --gate-modes: its one-unit /
                pairs tables separately),
  stream     -- debug knob gated = 0: inner launch + shell with pack / flag / unpack kernels on
                the comm stream (the round-4 overlapped pass),
  serial     -- overlap off: exchange, then the full pass.
--emulate-us adds the debug knob ipc_emulate_us (every exchange lasts at least that long: a
slower xGMI hop modelled on one GPU).

  python scripts/bench_gated.py --n 256 --k 3 --emulate-us 0 30 --out gpurun_out/gated.json
"""
import argparse
import dataclasses
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="+", default=[256], help="sub-domain edge (cells)")
    ap.add_argument("--k", type=int, nargs="+", default=[3])
    ap.add_argument("--passes", type=int, default=60)
    ap.add_argument("--emulate-us", type=float, nargs="+", default=[0.0, 30.0])
    ap.add_argument("--nbrs", nargs="+", default=["z", "plus", "all"])
    ap.add_argument("--prec", default="Float32")
    ap.add_argument("--out", default="")
    ap.add_argument("--gate-modes", type=int, nargs="+", default=[0],
                    help="debug knob gate_mode per gated row: 0 tuned (carried, one-unit and "
                         "pairs tables), 1 one-unit tables packed at the start only, 2 pairs "
                         "tables only, 3 carried one-unit tables only")
    ap.add_argument("--gated-only", action="store_true", help="skip the stream / serial rows")
    ap.add_argument("--stamps", action="store_true",
                    help="debug knob gate_stamps: the exchange's wall-clock stamps (after the "
                         "timed passes; the stamp resets add a copy per pass, so time without)")
    a = ap.parse_args()
    import torch  # noqa: F401
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    def settings(n, overlap):
        return Settings(L=n, precision=a.prec, F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                        noise=0.1, backend="AMDGPU", seed=77, overlap=overlap)

    def timed(sim, k):
        sim.init_fields()
        sim.randomize_fields(seed=5)
        sim.iterate(4 * k)  # warm-up (and first-use tuning)
        sim.synchronize()
        t0 = time.perf_counter()
        sim.iterate(a.passes * k)
        sim.synchronize()
        return 1e3 * (time.perf_counter() - t0) / a.passes

    def loop_dom(n, which):
        dom = init_domain(n, 1, 0, periodic=True)
        nbr = list(dom.nbr27)
        # index (dx + 1) * 9 + (dy + 1) * 3 + (dz + 1)
        if which == "z":  # keep dx = dy = 0
            nbr = [r if (i // 9 == 1 and (i // 3) % 3 == 1) or i == 13 else -1
                   for i, r in enumerate(nbr)]
        elif which == "plus":  # dx, dy, dz in {0, 1}: +x, +y, +z faces, their edges, the corner
            nbr = [r if i != 13 and i // 9 != 0 and (i // 3) % 3 != 0 and i % 3 != 0 else -1
                   for i, r in enumerate(nbr)]
        return dataclasses.replace(dom, periodic=False, nbr27=nbr)

    rows = []
    for n in a.n:
        for k in a.k:
            sim = GrayScott(settings(n, "auto"), init_domain(n, 1, 0), fuse=k)
            try:
                full = timed(sim, k)
            finally:
                sim.close()
            for which in a.nbrs:
                for em in a.emulate_us:
                    row = {"n": n, "k": k, "nbrs": which, "emulate_us": em,
                           "full_ms": round(full, 4)}
                    kinds = [(f"gated{m}" if len(a.gate_modes) > 1 else "gated", "on", 1, m)
                             for m in a.gate_modes]
                    if not a.gated_only:
                        kinds += [("stream", "on", 0, 0), ("serial", "off", 1, 0)]
                    for kind, ov, gated, mode in kinds:
                        native.debug_set("gated", gated)
                        native.debug_set("gate_mode", mode)
                        native.debug_set("ipc_emulate_us", em)
                        native.debug_set("gate_stamps", 1 if a.stamps else 0)
                        native.debug_set("ipc_pair_same_dir", 1 if which == "plus" else 0)
                        try:
                            sim = GrayScott(settings(n, ov), loop_dom(n, which), fuse=k,
                                            transport="ipc", loopback=True)
                            try:
                                ms = timed(sim, k)
                                row[kind + "_ms"] = round(ms, 4)
                                row[kind + "_x"] = round(ms / full, 4)
                                if kind.startswith("gated"):
                                    row[kind + "_ran"] = sim.gated
                                    row[kind + "_table"] = sim.engine.gate_info(k)
                                    row[kind + "_stamps_us"] = sim.engine.gate_stamps()
                            finally:
                                sim.close()
                        finally:
                            native.debug_set("gated", 1)
                            native.debug_set("ipc_emulate_us", 0)
                            native.debug_set("gate_stamps", 0)
                            native.debug_set("gate_mode", 0)
                            native.debug_set("ipc_pair_same_dir", 0)
                    rows.append(row)
                    print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(rows, fh, indent=1)


if __name__ == "__main__":
    main()
