# Fuse depth T=2 vs T=3 on small grids with the round-2 kernel (pipeline-fill skip), bench.py, one MI355X.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-fuse_small}
mkdir -p $O
cd $R
for rep in 1 2; do
for L in 64 96 128 192 256; do
  st=$((2000 * 64 / L)); [ $st -lt 300 ] && st=300
  for f in 2 3; do
    timeout -k 10 120 python bench.py --L $L --fuse $f --steps $st --warmup 30 > $O/tmp.json 2>> $O/err.txt || { echo "bench failed L=$L f=$f"; exit 1; }
    python -c "import json; r=json.loads(open('$O/tmp.json').read()); print('L=%d fuse=%d steps=%d MLUPS=%.0f us/step=%.2f kernel=%s' % ($L, $f, r['steps'], r['value'], r['ms_per_step']*1e3, r['config']['fused_kernel']))" | tee -a $O/fuse.txt
  done
done
done
