#!/bin/bash
# Refresh-priced planner: GPU tests, then the driver's command A/B (plan_fill 1 vs 0), interleaved.
set -o pipefail
O=gpurun_out/r6pf
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_planner.py tests/test_gpu_oracle.py -k "planner or planned or refresh" \
  -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed|refresh" $O/tests.log | tail -6
for r in 1 2 3; do
  for f in 1 0; do
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --debug-knob plan_fill=$f > $O/b_${r}_$f.json 2> $O/b_${r}_$f.err || { tail -20 $O/b_${r}_$f.err; exit 1; }
    python - "$O/b_${r}_$f.json" $f <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = r["config"]
print(f"plan_fill={sys.argv[2]} {r['value']:,.0f} MLUPS {r['ms_per_step']} ms/step plan {c.get('pass_plan')} fill {c.get('bc_fill_ms')} golden {r.get('check', {}).get('golden_ok')}")
PY
  done
done
