#!/bin/bash
# Outer-ghost refresh at the end of each advance() + refresh-priced planner: GPU tests that run
# the planned / phased / oracle paths, three driver commands, and the kernel timeline of one.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6eb
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_planner.py tests/test_gpu_oracle.py tests/test_gpu_phases.py tests/test_gpu_block.py \
  -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -3
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$r.json 2> $O/b_$r.err || { tail -20 $O/b_$r.err; exit 1; }
  python - "$O/b_$r.json" <<'PY'
import json, sys
r = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
c = r["config"]
print(f"{r['value']:,.0f} MLUPS {r['ms_per_step']} ms/step plan {c.get('pass_plan')} fill {c.get('bc_fill_ms')} golden {r.get('check', {}).get('golden_ok')}")
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bt.json 2> $O/bt.err || { tail -20 $O/bt.err; exit 1; }
python3 scripts/trace_window.py $O/trace > $O/timeline.txt || exit 1
cat $O/timeline.txt
tail -1 $O/bt.json | cut -c1-200
