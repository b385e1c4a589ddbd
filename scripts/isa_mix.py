#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc --save-temps assembly file.

  hipcc -O3 -std=c++17 --offload-arch=gfx950 -Icsrc/include -c csrc/hip/inst/fused_float.hip \
        --save-temps -o /tmp/ff.o
  python scripts/isa_mix.py fused_float-hip-amdgcn-amd-amdhsa-gfx950.s Li3ELi4ELi12ELi2ELb0ELb1ELb1ELb1ELi0E

Prints the instruction counts of the kernel whose symbol contains the given substring, and
the VALU count of its steady-state loop body (the largest basic-block cycle: the last
backward branch's target to the branch).
"""
import collections
import re
import sys


def body_of(asm: str, key: str) -> str:
    names = re.findall(r"^(_Z\S*):", asm, re.M)
    hits = [n for n in names if key in n]
    if len(hits) != 1:
        raise SystemExit(f"{len(hits)} kernels match {key!r}: {hits[:4]}")
    start = asm.index(hits[0] + ":")
    end = asm.index(".Lfunc_end", start)
    return asm[start:end]


def mix(lines):
    ops = collections.Counter()
    for line in lines:
        t = line.strip()
        if not t or t.startswith((".", ";", "_")) or t.endswith(":"):
            continue
        ops[t.split()[0]] += 1
    return ops


def main():
    asm = open(sys.argv[1]).read()
    body = body_of(asm, sys.argv[2])
    lines = body.split("\n")
    ops = mix(lines)
    print("static total VALU", sum(v for k, v in ops.items() if k.startswith("v_")),
          "SALU", sum(v for k, v in ops.items() if k.startswith("s_")))
    # the largest loop: a backward s_cbranch / s_branch to a label above it
    labels = {l.strip()[:-1]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\S+:$", l.strip())}
    best = None
    for i, l in enumerate(lines):
        m = re.match(r"\s*s_(cbranch_\w+|branch)\s+(\.LBB\S+)", l)
        if m and m.group(2) in labels and labels[m.group(2)] < i:
            n = i - labels[m.group(2)]
            if best is None or n > best[1] - best[0]:
                best = (labels[m.group(2)], i)
    if best:
        lops = mix(lines[best[0]:best[1] + 1])
        print(f"largest loop: lines {best[0]}-{best[1]}, VALU",
              sum(v for k, v in lops.items() if k.startswith("v_")))
        for k, v in lops.most_common(40):
            print(f"{v:6d} {k}")


if __name__ == "__main__":
    main()
