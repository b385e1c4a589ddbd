# Round 6 sweep: the driver's command, BASELINE config 2 (L=256, 1000 steps), L=64 / 1024, and the
# multi-rank rehearsal on one card (link probe + model table)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6s}
mkdir -p $O
cd $R
row() { python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print(sys.argv[2], d['value'], d['ms_per_step'], c.get('pass_plan', [])[:8], len(c.get('pass_plan', [])), {k: (v['tile'], v['sched'], v['ms']) for k, v in c['fused_kernel'].items()}, d['check'].get('golden_ok'))" "$@" | tee -a $O/summary.txt; }
for i in 1 2; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/k20_$i.json 2> $O/k20_$i.err || exit 1
  row $O/k20_$i.json "L512 K20" || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --L 256 --steps 1000 --warmup 100 > $O/l256_$i.json 2> $O/l256_$i.err || exit 1
  row $O/l256_$i.json "L256 K1000" || exit 1
done
timeout -k 10 300 python bench.py --gpus 1 --L 64 --steps 2000 --warmup 100 > $O/l64.json 2> $O/l64.err || exit 1
row $O/l64.json "L64 K2000" || exit 1
timeout -k 10 300 python bench.py --gpus 1 --L 1024 --steps 40 --warmup 4 > $O/l1024.json 2> $O/l1024.err || exit 1
row $O/l1024.json "L1024 K40" || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 400 --warmup 5 > $O/k400.json 2> $O/k400.err || exit 1
row $O/k400.json "L512 K400" || exit 1
for n in 2 4; do
  timeout -k 10 400 python bench.py --gpus $n --steps 20 --warmup 5 > $O/b$n.json 2> $O/b$n.err || { tail -20 $O/b$n.err; exit 1; }
  python scripts/rehearsal_row.py $O/b$n.json | tee -a $O/rehearsal.txt
done
timeout -k 10 500 python bench.py --gpus 8 --steps 20 --warmup 5 --debug-knob gated=2 > $O/b8g.json 2> $O/b8g.err || { tail -20 $O/b8g.err; exit 1; }
python scripts/rehearsal_row.py $O/b8g.json | tee -a $O/rehearsal.txt
