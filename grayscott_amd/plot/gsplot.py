"""Slice plots of a Gray-Scott output stream (the reference's src/plot/gdsplot.jl is an empty
placeholder; this provides what the ADIOS2-Examples ``gsplot`` does, without matplotlib).

    python -m grayscott_amd.plot.gsplot gs.bp --var V --step -1 --axis z --index mid -o v.png

Writes an 8-bit PNG (PIL) of one axis-aligned slice with a built-in colour map, or a
whole-stream montage with ``--all``.
"""
from __future__ import annotations

import argparse
import sys
from typing import Optional, Sequence

import numpy as np

from ..io.bp4 import BP4Reader

# compact "viridis-like" colour map: 5 anchor colours, linearly interpolated
_ANCHORS = np.array([[68, 1, 84], [59, 82, 139], [33, 145, 140], [94, 201, 98], [253, 231, 37]],
                    dtype=np.float64)


def colormap(x: np.ndarray) -> np.ndarray:
    x = np.clip(x, 0.0, 1.0) * (len(_ANCHORS) - 1)
    i = np.minimum(x.astype(np.int64), len(_ANCHORS) - 2)
    f = (x - i)[..., None]
    return ((1 - f) * _ANCHORS[i] + f * _ANCHORS[i + 1]).astype(np.uint8)


def read_slice(path: str, var: str = "V", step: int = -1, axis: str = "z",
               index: Optional[int] = None) -> np.ndarray:
    with BP4Reader(path) as r:
        Lz, Ly, Lx = r.variables(step if step >= 0 else r.steps + step)[var].shape
        n = {"z": Lz, "y": Ly, "x": Lx}[axis]
        idx = n // 2 if index is None else int(index)
        if axis == "z":
            return r.read(var, step, (idx, 0, 0), (1, Ly, Lx))[0]
        if axis == "y":
            return r.read(var, step, (0, idx, 0), (Lz, 1, Lx))[:, 0, :]
        return r.read(var, step, (0, 0, idx), (Lz, Ly, 1))[:, :, 0]


def to_image(a: np.ndarray, vmin: Optional[float] = None, vmax: Optional[float] = None,
             scale: int = 4):
    from PIL import Image
    lo = float(a.min()) if vmin is None else vmin
    hi = float(a.max()) if vmax is None else vmax
    norm = (a - lo) / (hi - lo) if hi > lo else np.zeros_like(a, dtype=np.float64)
    rgb = colormap(norm)[::-1]  # origin at the bottom
    img = Image.fromarray(rgb, mode="RGB")
    if scale > 1:
        img = img.resize((img.width * scale, img.height * scale), Image.NEAREST)
    return img


def main(args: Optional[Sequence[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="gs-plot", description=__doc__.split("\n")[0])
    p.add_argument("input")
    p.add_argument("--var", default="V", choices=["U", "V"])
    p.add_argument("--step", type=int, default=-1)
    p.add_argument("--axis", default="z", choices=["x", "y", "z"])
    p.add_argument("--index", type=int, default=None)
    p.add_argument("--scale", type=int, default=4)
    p.add_argument("--all", action="store_true", help="montage of every step")
    p.add_argument("-o", "--output", default="gsplot.png")
    ns = p.parse_args(sys.argv[1:] if args is None else args)
    if ns.all:
        from PIL import Image
        with BP4Reader(ns.input) as r:
            nsteps = r.steps
        slices = [read_slice(ns.input, ns.var, s, ns.axis, ns.index) for s in range(nsteps)]
        lo = min(float(s.min()) for s in slices)
        hi = max(float(s.max()) for s in slices)
        imgs = [to_image(s, lo, hi, ns.scale) for s in slices]
        cols = int(np.ceil(np.sqrt(len(imgs))))
        rows = int(np.ceil(len(imgs) / cols))
        w, h = imgs[0].size
        sheet = Image.new("RGB", (cols * w, rows * h))
        for i, im in enumerate(imgs):
            sheet.paste(im, ((i % cols) * w, (i // cols) * h))
        sheet.save(ns.output)
    else:
        to_image(read_slice(ns.input, ns.var, ns.step, ns.axis, ns.index), scale=ns.scale).save(ns.output)
    print(ns.output)
    return 0


if __name__ == "__main__":
    sys.exit(main())
