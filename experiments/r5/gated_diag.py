"""Where a gated loopback pass differs from the self-copy reference (diagnostic, one GPU).

  python experiments/r5/gated_diag.py --L 40 --k 3 --steps 3
"""
import argparse
import dataclasses
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--L", type=int, default=40)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--steps", type=int, nargs="+", default=[3, 6, 16])
    ap.add_argument("--which", default="all")
    ap.add_argument("--noise", type=float, default=0.1)
    a = ap.parse_args()
    import torch  # noqa: F401
    from grayscott_amd.models.grayscott import GrayScott
    from grayscott_amd.ops import native
    from grayscott_amd.parallel.decomp import init_domain
    from grayscott_amd.utils.config import Settings

    dom = init_domain(a.L, 1, 0, periodic=True)
    nbr = list(dom.nbr27)
    if a.which == "z":
        nbr = [r if (i // 9 == 1 and (i // 3) % 3 == 1) or i == 13 else -1 for i, r in enumerate(nbr)]
    elif a.which == "x":
        nbr = [r if (i % 3 == 1 and (i // 3) % 3 == 1) or i == 13 else -1 for i, r in enumerate(nbr)]
    elif a.which == "y":
        nbr = [r if (i % 3 == 1 and i // 9 == 1) or i == 13 else -1 for i, r in enumerate(nbr)]
    loop = dataclasses.replace(dom, periodic=False, nbr27=nbr)
    s = Settings(L=a.L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                 noise=a.noise, backend="AMDGPU", seed=99, overlap="on")

    def run(steps, gated, **kw):
        native.debug_set("gated", gated)
        sim = GrayScott(s, loop, fuse=a.k, **kw)
        try:
            sim.init_fields()
            sim.randomize_fields(seed=7)
            sim.iterate(steps)
            sim.synchronize()
            u, v = sim.get_fields()
            return u, v, sim.gated, sim.engine.gate_info(a.k)
        finally:
            sim.close()
            native.debug_set("gated", 1)

    for steps in a.steps:
        u0, v0, _, _ = run(steps, 1)
        us, vs, gs_, _ = run(steps, 0, transport="ipc", loopback=True)
        ug, vg, gg, info = run(steps, 1, transport="ipc", loopback=True)
        for name, u, g in (("stream", us, gs_), ("gated", ug, gg)):
            bad = u != u0
            rec = {"steps": steps, "kind": name, "gated": g, "bad": int(bad.sum()), "of": int(bad.size)}
            if name == "gated":
                rec["gate"] = info
            if bad.any():
                zz, yy, xx = np.nonzero(bad)
                rec["z"] = np.bincount(zz, minlength=a.L).tolist()
                rec["y"] = np.bincount(yy, minlength=a.L).tolist()
                rec["x"] = np.bincount(xx, minlength=a.L).tolist()
                rec["first"] = [int(zz[0]), int(yy[0]), int(xx[0])]
                rec["maxdiff"] = float(np.abs(u - u0).max())
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
