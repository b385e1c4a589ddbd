import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from tests.mp_utils import run_ranks

def cfg(L, steps, fuse, overlap, dims, transport="host"):
    c = {"settings": dict(L=L, precision="Float32", F=0.02, k=0.048, dt=1.0, Du=0.2, Dv=0.1,
                          noise=0.1, backend="AMDGPU", periodic=False, seed=1234, overlap=overlap),
         "steps": steps, "fuse": fuse, "transport": transport}
    if dims: c["dims"] = dims
    return c

def main():
  for (world, dims, L, fuse, ov) in [(8, [1,2,4], 64, 2, "on"), (8, [1,2,4], 64, 2, "off"), (8, [1,2,4], 64, 3, "on"),
                                      (4, [1,2,2], 64, 2, "on"), (4, [1,1,4], 64, 2, "on"), (8,[1,1,8],64,2,"on"),
                                      (4, [2,2,1], 64, 2, "on"), (4, [1,4,1], 64, 2, "on")]:
      steps = 11
      u1, v1, _ = run_ranks(1, cfg(L, steps, fuse, "off", None))
      un, vn, meta = run_ranks(world, cfg(L, steps, fuse, ov, dims))
      bad = np.argwhere(un != u1)
      zs = sorted(set(bad[:, 0].tolist()))[:20] if len(bad) else []
      ys = sorted(set(bad[:, 1].tolist()))[:40] if len(bad) else []
      print(world, dims, L, fuse, ov, "overlapped", all(m["overlapped"] for m in meta), "mismatch", len(bad), "z", zs, "y", ys, flush=True)


if __name__ == "__main__":
    main()
