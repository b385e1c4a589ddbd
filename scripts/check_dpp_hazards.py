#!/usr/bin/env python3
"""Check the built gfx950 code object for VALU-write -> DPP-read hazards.

A DPP instruction reading a VGPR (its src0) needs 2 wait states after a VALU instruction that
wrote that VGPR (CDNA3/4 ISA, "manually inserted wait states").  The compiler inserts them for
the DPP it generates, but not around inline asm: the fused kernel's x-neighbour sums
(csrc/hip/fused.hpp, lane_pair_sum_add) are written as asm without the leading `s_nop`,
relying on their operands coming from loads or from earlier pipeline iterations.  This script
proves that property on the shipped binary: it extracts the gfx950 code object from
libgs_hip.so, disassembles it, and walks back from every DPP instruction counting wait states
(each instruction 1, `s_nop N` N+1) until 2 are covered.  A VALU write of the DPP source inside
that window, or a branch target inside it (a path the linear walk does not see), fails; so
does an EXEC write within 5 wait states.  Only the DPP source operand (src0) is checked: the
lane permutation applies to src0 alone, and the two-instruction pattern "DPP op t <- f(v);
DPP op r <- g(v, t)" (t read as a plain src1 right after it is written) has produced bit-exact
results since round 1 (the compiler's own rule, which also covers src1, is more conservative).

  python scripts/check_dpp_hazards.py [grayscott_amd/_lib/libgs_hip.so]   # exit 1 on a hazard
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fatbin import LLVM, code_objects  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_INSN = re.compile(r"^\s+([a-z_0-9]+)\s*(.*?)\s*//\s*([0-9A-F]{12}):")
_BRANCH = re.compile(r"^s_(c?branch\w*|call\w*)$")
_VREG = re.compile(r"^v(\d+)$|^v\[(\d+):(\d+)\]$")


def disassemble(lib: str) -> list[str]:
    """One disassembly per code object (addresses restart in each, so they are checked apart)."""
    with tempfile.TemporaryDirectory() as d:
        return [subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], check=True,
                               capture_output=True, text=True).stdout
                for co in code_objects(lib, d)]


def check_all(texts: list[str]):
    checked, problems = 0, []
    for t in texts:
        n, p = check(t)
        checked, problems = checked + n, problems + p
    return checked, problems


def vregs(op: str):
    m = _VREG.match(op.strip())
    if not m:
        return set()
    if m.group(1) is not None:
        return {int(m.group(1))}
    return set(range(int(m.group(2)), int(m.group(3)) + 1))


def check(text: str):
    """Returns (number of DPP instructions checked, list of problems)."""
    insns = []  # (addr, mnemonic, operands)
    targets = set()
    for line in text.splitlines():
        m = _INSN.match(line)
        if not m:
            continue
        mn, ops, addr = m.group(1), m.group(2), int(m.group(3), 16)
        insns.append((addr, mn, ops))
        if _BRANCH.match(mn):
            tm = re.search(r"\b(\d+)\b", ops.split("//")[0]) if mn.startswith("s_") else None
            if tm is not None:
                # relative simm16 in dwords from the next instruction (4-byte s_branch encoding)
                off = int(tm.group(1))
                off = off - 0x10000 if off >= 0x8000 else off
                targets.add(addr + 4 + 4 * off)
    checked, problems = 0, []
    for i, (addr, mn, ops) in enumerate(insns):
        if "_dpp" not in mn and "dpp" not in ops:
            continue
        if not mn.startswith("v_"):
            continue
        parts = [p.strip() for p in ops.split(",")]
        if len(parts) < 2:
            continue
        src = vregs(parts[1])
        if not src:
            continue
        checked += 1
        ws = 0
        j = i - 1
        if addr in targets:
            problems.append(f"{addr:#x} {mn} {ops[:60]}: branch target (unchecked path)")
            continue
        # EXEC written within 5 wait states before a DPP instruction (the compiler's rule)
        ew, k = 0, i - 1
        while ew < 5 and k >= 0:
            _, emn, eops = insns[k]
            dst0 = eops.split(",")[0].strip()
            if dst0.startswith("exec") or emn.startswith("v_cmpx") or "saveexec" in emn:
                problems.append(f"{addr:#x} {mn}: EXEC written by {emn} {ew} wait state(s) before")
                break
            if emn == "s_nop":
                n = re.match(r"\s*(0x[0-9a-f]+|\d+)", eops)
                ew += (int(n.group(1), 0) if n else 0) + 1
            else:
                ew += 1
            k -= 1
        while ws < 2 and j >= 0:
            paddr, pmn, pops = insns[j]
            if pmn.startswith("v_") and not pmn.startswith(("v_cmp", "v_readlane",
                                                              "v_readfirstlane")):
                dst = vregs(pops.split(",")[0])
                if dst & src:
                    problems.append(f"{addr:#x} {mn} reads v{sorted(dst & src)} written by "
                                    f"{pmn} at {paddr:#x} with {ws} wait state(s)")
                    break
            if pmn == "s_nop":
                n = re.match(r"\s*(0x[0-9a-f]+|\d+)", pops)
                ws += (int(n.group(1), 0) if n else 0) + 1
            else:
                ws += 1
            if paddr in targets and ws < 2:
                problems.append(f"{addr:#x} {mn}: branch target {paddr:#x} inside the window")
                break
            j -= 1
    return checked, problems


def main(argv):
    lib = argv[1] if len(argv) > 1 else os.path.join(ROOT, "grayscott_amd", "_lib", "libgs_hip.so")
    checked, problems = check_all(disassemble(lib))
    for p in problems[:50]:
        print("HAZARD", p)
    print(f"{os.path.basename(lib)}: {checked} DPP instructions checked, {len(problems)} hazard(s)")
    return 1 if problems or checked == 0 else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
