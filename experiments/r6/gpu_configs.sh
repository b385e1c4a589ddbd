#!/bin/bash
# Final tree: BASELINE configs on one GPU -- L=256 1000 steps (config 2), L=1024 fp64 (config 4's
# precision and size), L=512 fp64, L=512 400 steps.
set -o pipefail
O=gpurun_out/r6cfg
mkdir -p $O
run() {
  local tag=$1; shift
  timeout -k 10 400 python bench.py --gpus 1 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  python - $O/$tag.json $tag <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = r["config"]
print(f"{sys.argv[2]}: {r['value']:,.1f} MLUPS {r['ms_per_step']} ms/step plan {sorted(set(c.get('pass_plan') or []))} x{len(c.get('pass_plan') or [])} kernels {c.get('fused_kernel')} golden {r.get('check', {}).get('golden_ok')}")
PY
}
run l256_1000 --L 256 --steps 1000 --warmup 100
run l1024_f64 --L 1024 --precision Float64 --steps 60 --warmup 6
run l512_f64 --L 512 --precision Float64 --steps 60 --warmup 6
run l512_400 --steps 400 --warmup 40
