# Round 6: fp64 LDS ring (4x8:1sl) after the padding-store fix: golden
# repeats, bitwise vs the register ring, the fp32 LR shapes' bitwise check, then timings
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6f}
mkdir -p $O
cd $R
GOLD=1 REPS=6 CFGS=4x8:1s,4x8:1sl,4x8:1sl timeout -k 10 300 python -u experiments/r6/f64_lr_diag.py > $O/gold.txt 2>&1 || { cat $O/gold.txt; exit 1; }
cat $O/gold.txt
timeout -k 10 300 python -u experiments/r6/lr_check.py --check-only > $O/lr_check.txt 2>&1 || { tail -30 $O/lr_check.txt; exit 1; }
tail -2 $O/lr_check.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "fp64_lds_ring" -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 600 python -u experiments/r6/f64_ab.py > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
for L in 512 1024; do
  timeout -k 10 300 python bench.py --gpus 1 --L $L --precision Float64 --steps 60 --warmup 6 > $O/b$L.json 2> $O/b$L.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('L=', c['L'], d['value'], d['ms_per_step'], c['pass_plan'], c['fused_kernel'], d['check'].get('golden_ok'))" $O/b$L.json | tee -a $O/summary.txt
done
