# Round 6: the driver's K=20 window by pass order / depth mix, interleaved on one box
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6o}
mkdir -p $O
cd $R
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], d['value'], d['ms_per_step'], c.get('pass_plan'), d['check'].get('golden_ok'))" "$@" | tee -a $O/summary.txt; }
for r in 1 2 3 4; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/a$r.json 2>/dev/null || exit 1
  row $O/a$r.json "deepest-first" || exit 1
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --debug-knob plan_order=1 > $O/b$r.json 2>/dev/null || exit 1
  row $O/b$r.json "shallowest-first" || exit 1
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --fuse 4 > $O/c$r.json 2>/dev/null || exit 1
  row $O/c$r.json "T=4 x5" || exit 1
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --fuse 3 > $O/d$r.json 2>/dev/null || exit 1
  row $O/d$r.json "T=3 greedy (r5)" || exit 1
done
