"""``bpls``-like listing of a BP4 file (ADIOS2's bpls is not available here).

    python -m grayscott_amd.io.bpls gs.bp            # variables, shapes, min/max
    python -m grayscott_amd.io.bpls gs.bp -a         # + attributes
    python -m grayscott_amd.io.bpls gs.bp -D         # + per-block decomposition
    python -m grayscott_amd.io.bpls gs.bp -d step    # dump a variable
"""
from __future__ import annotations

import argparse
import sys
from typing import Optional, Sequence

import numpy as np

from .bp4 import BP4Reader

_TYPES = {0: "int8_t", 1: "int16_t", 2: "int32_t", 4: "int64_t", 5: "float", 6: "double",
          9: "string", 12: "string array", 50: "uint8_t", 51: "uint16_t", 52: "uint32_t",
          54: "uint64_t"}


def listing(path: str, attrs: bool = False, decomp: bool = False) -> str:
    lines = []
    with BP4Reader(path) as r:
        names = {}
        for s in range(r.steps):
            for n, vi in r.variables(s).items():
                names.setdefault(n, []).append((s, vi))
        for n, occ in names.items():
            vi = occ[0][1]
            mins = [b.vmin if b.vmin is not None else b.value for _, v in occ for b in v.blocks]
            maxs = [b.vmax if b.vmax is not None else b.value for _, v in occ for b in v.blocks]
            shape = "scalar" if vi.is_single_value else "{" + ", ".join(str(d) for d in vi.shape) + "}"
            lines.append(f"  {_TYPES.get(vi.type, vi.type):10s} {n:20s} {len(occ)}*{shape} = "
                         f"{min(mins):.6g} / {max(maxs):.6g}")
            if decomp:
                for s, v in occ:
                    for i, b in enumerate(v.blocks):
                        lines.append(f"        step {s:4d} block {i:3d}: [{', '.join(f'{o}:{o + c - 1}' for o, c in zip(b.start, b.count))}]"
                                     f" = {b.vmin if b.vmin is not None else b.value} / "
                                     f"{b.vmax if b.vmax is not None else b.value}  (data.{b.file_index})")
        if attrs:
            for k, v in r.attributes.items():
                if isinstance(v, np.ndarray):
                    v = v.tolist()
                lines.append(f"  attr {k:28s} = {v!r}")
    return "\n".join(lines)


def main(args: Optional[Sequence[str]] = None) -> int:
    p = argparse.ArgumentParser(prog="gs-bpls")
    p.add_argument("file")
    p.add_argument("-a", "--attrs", action="store_true")
    p.add_argument("-D", "--decomp", action="store_true")
    p.add_argument("-d", "--dump", default=None)
    ns = p.parse_args(sys.argv[1:] if args is None else args)
    print(listing(ns.file, ns.attrs, ns.decomp))
    if ns.dump:
        with BP4Reader(ns.file) as r:
            for s in range(r.steps):
                print(f"step {s}: {r.read(ns.dump, s)}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
