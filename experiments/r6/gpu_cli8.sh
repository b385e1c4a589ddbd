#!/bin/bash
# BASELINE config 3's example through the CLI with 8 ranks on ONE GPU (IPC transport: RCCL refuses
# several ranks per device): 60 steps, one output step, then the BP4 file read back.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6cli8
mkdir -p $O && cd $O
sed -e 's/^steps = .*/steps = 60/' -e 's/^plotgap = .*/plotgap = 60/' -e 's/^transport = .*/transport = "ipc"/' \
  $R/examples/l512-2x2x2.toml > run.toml
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29555 $R/gray-scott.py run.toml > run.log 2>&1 || { tail -40 run.log; exit 1; }
tail -4 run.log
tail -1 perf-512L-2x2x2.jsonl | cut -c1-600
timeout -k 10 200 python - <<'PY' || { rm -rf gs-512L-F32-2x2x2.bp; exit 1; }
import os, sys
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import numpy as np
from grayscott_amd.io import bp4
with bp4.BP4Reader("gs-512L-F32-2x2x2.bp") as r:
    print("steps", r.steps, "vars", sorted(r.variables(0)))
    u = r.read("U", step=-1)
    v = r.read("V", step=-1)
    print("U", u.shape, u.dtype, float(u.min()), float(u.max()), float(u.mean()),
          "V", float(v.min()), float(v.max()), float(v.mean()), "finite", bool(np.isfinite(u).all()))
PY
ls -la gs-512L-F32-2x2x2.bp | head
rm -rf gs-512L-F32-2x2x2.bp
