# Round 3: small grids -- fuse depth 1 (the single-step kernel every step) vs 2 (the fused kernel).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-smallf3}
mkdir -p $O
cd $R
for L in 64 96 128; do
  for f in 1 2; do
    timeout -k 10 120 python bench.py --L $L --steps 2000 --warmup 200 --fuse $f > $O/l${L}_f$f.json 2>> $O/err.txt || { echo "failed L=$L fuse=$f"; exit 1; }
    python3 -c "import json; r=json.load(open('$O/l${L}_f$f.json')); print('L=$L fuse=$f', r['value'], r['ms_per_step'], r['check'].get('max_abs_err'))" | tee -a $O/summary.txt
  done
done
