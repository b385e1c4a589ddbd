# Round 6: LDS-ring shapes + T=4 bitwise/timings, then the driver's bench command with the planner
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6d}
mkdir -p $O
cd $R
timeout -k 10 400 python -u experiments/r6/lr_check.py --rounds 2 --cases 3:4x12:1s 3:4x12:2s 3:4x12:1sfl 4:4x12:1sl 4:4x12:1sfl 2:4x12:1s 2:4x12:2sl > $O/lr.txt 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_$i.json 2> $O/b20_$i.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('K=20', d['value'], d['ms_per_step'], c['pass_plan'], c['fused_kernel'], d['check'].get('golden_ok'))" $O/b20_$i.json | tee -a $O/summary.txt
done
timeout -k 10 200 python bench.py --gpus 1 --steps 400 --warmup 5 > $O/b400.json 2> $O/b400.err || exit 1
python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('K=400', d['value'], d['ms_per_step'], c['pass_plan'][:3], len(c['pass_plan']), c['fused_kernel'])" $O/b400.json | tee -a $O/summary.txt
