"""Would hipGraph replay shorten the engine's steps?  advance(n) enqueued as usual vs captured once
and replayed (csrc/hip/backend_hip.hip gs_graph_probe; timing only -- replays repeat a time step)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
from grayscott_amd.models.grayscott import GrayScott  # noqa: E402
from grayscott_amd.ops import native  # noqa: E402
from grayscott_amd.parallel.decomp import init_domain  # noqa: E402
from grayscott_amd.utils.config import Settings  # noqa: E402

lib = native.load("hip")
lib.gs_graph_probe.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_int32,
                               ctypes.POINTER(ctypes.c_double)]
lib.gs_graph_probe.restype = ctypes.c_int
for L, n, reps in [(64, 10, 300), (64, 100, 30), (96, 10, 200), (128, 10, 200), (256, 20, 20), (512, 20, 5)]:
    s = Settings(L=L, precision="Float32", noise=0.1, backend="AMDGPU", seed=2024,
                 F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1)
    side = torch.cuda.Stream()  # the legacy default stream cannot be captured
    with torch.cuda.stream(side):
        sim = GrayScott(s, init_domain(L, 1, 0))
    try:
        sim.init_fields()
        plan = sim.engine.plan_passes(n)
        out = (ctypes.c_double * 2)()
        rc = lib.gs_graph_probe(sim.engine.h, 0, n, reps, out)
        if rc != 0:
            print(f"L={L}: probe failed: {native.last_error(lib)}")
            break
        e, g = out[0], out[1]
        print(f"L={L:4d} n={n:3d} plan {plan or sim.depth} choice {sim.fused_choice()}: "
              f"stream {e:.3f} us/step ({L**3 / e:,.0f} MLUPS)  graph {g:.3f} us/step "
              f"({L**3 / g:,.0f} MLUPS)  graph/stream {g / e:.3f}", flush=True)
    finally:
        sim.close()
