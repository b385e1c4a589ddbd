# Round 6: single-GPU rate across grid sizes (fp32, random init, the planner's passes)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6w}
mkdir -p $O
cd $R
for L in 128 192 256 320 384 448 512 640 768 896 1024; do
  n=$(( 200 * 512 * 512 * 512 / (L * L * L) )); [ $n -gt 2000 ] && n=2000; [ $n -lt 40 ] && n=40
  timeout -k 10 300 python bench.py --gpus 1 --L $L --steps $n --warmup 10 > $O/L$L.json 2> $O/L$L.err || { tail -5 $O/L$L.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; pl=c.get('pass_plan', []); print(f\"L={c['L']:5d} steps={d['steps']:5d} {d['value']:10.1f} MLUPS {d['ms_per_step']:.5f} ms/step depths={sorted(set(pl))} passes={len(pl)} \" + ' '.join(f\"T{k}:{v['tile']}/s{v['sched']}/{v['ms']}\" for k, v in c['fused_kernel'].items()) + f\" golden={d['check'].get('golden_ok')}\")" $O/L$L.json | tee -a $O/summary.txt
done
