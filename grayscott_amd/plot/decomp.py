"""Decomposition viewer (the reference's src/plot/decomp.jl is an empty placeholder; the
ADIOS2-Examples ``decomp`` plots which rank owns which block).

    python -m grayscott_amd.plot.decomp 512 8            # table of rank blocks
    python -m grayscott_amd.plot.decomp --from gs.bp     # blocks actually written to a file
    python -m grayscott_amd.plot.decomp 64 6 --png d.png # z-mid slice coloured by owner rank
"""
from __future__ import annotations

import argparse
import sys
from typing import List, Optional, Sequence, Tuple

import numpy as np

from ..io.bp4 import BP4Reader
from ..parallel.decomp import all_domains


def blocks_from_domains(L: int, nprocs: int, periodic: bool = False):
    out = []
    for d in all_domains(L, nprocs, periodic):
        out.append({"rank": d.rank, "coords": d.coords, "start_xyz": tuple(d.proc_offsets),
                    "count_xyz": tuple(d.proc_sizes), "neighbors": d.proc_neighbors})
    return out


def blocks_from_file(path: str, var: str = "U", step: int = 0):
    with BP4Reader(path) as r:
        vi = r.variables(step)[var]
        out = []
        for b in vi.blocks:
            # row-major (z, y, x) -> (x, y, z)
            out.append({"rank": b.file_index, "start_xyz": tuple(reversed(b.start)),
                        "count_xyz": tuple(reversed(b.count)), "min": b.vmin, "max": b.vmax})
        return out, vi.shape


def owner_slice(blocks, L: Tuple[int, int, int], z: int) -> np.ndarray:
    own = np.full((L[1], L[0]), -1, dtype=np.int64)
    for b in blocks:
        (x0, y0, z0), (nx, ny, nz) = b["start_xyz"], b["count_xyz"]
        if z0 <= z < z0 + nz:
            own[y0:y0 + ny, x0:x0 + nx] = b["rank"]
    return own


def main(args: Optional[Sequence[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="gs-decomp", description=__doc__.split("\n")[0])
    p.add_argument("L", nargs="?", type=int)
    p.add_argument("nprocs", nargs="?", type=int)
    p.add_argument("--from", dest="path", default=None, help="read the blocks of a BP4 file")
    p.add_argument("--periodic", action="store_true")
    p.add_argument("--png", default=None)
    ns = p.parse_args(sys.argv[1:] if args is None else args)
    if ns.path:
        blocks, shape = blocks_from_file(ns.path)
        L = (shape[2], shape[1], shape[0])
    else:
        if ns.L is None or ns.nprocs is None:
            p.error("L and nprocs are required without --from")
        blocks = blocks_from_domains(ns.L, ns.nprocs, ns.periodic)
        L = (ns.L, ns.L, ns.L)
    print(f"global extent (x,y,z) = {L}, {len(blocks)} blocks")
    for b in blocks:
        extra = f" neighbours={b['neighbors']}" if "neighbors" in b else ""
        print(f"  rank {b['rank']:4d} start={b['start_xyz']} count={b['count_xyz']}{extra}")
    if ns.png:
        from PIL import Image
        own = owner_slice(blocks, L, L[2] // 2)
        n = max(1, len(blocks))
        rng = np.random.default_rng(7)
        pal = rng.integers(40, 255, size=(n + 1, 3), dtype=np.uint8)
        img = pal[np.where(own < 0, n, own)][::-1]
        Image.fromarray(img, mode="RGB").resize((L[0] * 4, L[1] * 4), Image.NEAREST).save(ns.png)
        print(ns.png)
    return 0


if __name__ == "__main__":
    sys.exit(main())
