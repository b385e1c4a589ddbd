"""Extract the gfx950 code objects from a built HIP shared library (no GPU needed).

The library links several translation units (csrc/hip/backend_hip.hip + csrc/hip/inst/*.hip),
so its .hip_fatbin section holds one offload bundle per unit, back to back; each is unbundled
separately.
"""
from __future__ import annotations

import os
import subprocess

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib: str, workdir: str) -> list[str]:
    """Writes every gfx950 code object of `lib` into `workdir`; returns their paths."""
    fat = os.path.join(workdir, "fatbin")
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fat}", lib], check=True)
    with open(fat, "rb") as f:
        data = f.read()
    starts = []
    i = data.find(_MAGIC)
    while i >= 0:
        starts.append(i)
        i = data.find(_MAGIC, i + 1)
    out = []
    for k, s in enumerate(starts):
        part = os.path.join(workdir, f"bundle{k}")
        with open(part, "wb") as f:
            f.write(data[s:starts[k + 1] if k + 1 < len(starts) else len(data)])
        co = os.path.join(workdir, f"gfx950_{k}.co")
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                        f"--input={part}", f"--targets={TARGET}", f"--output={co}"], check=True)
        out.append(co)
    return out
