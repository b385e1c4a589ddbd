# Round 3: fp64 fuse depth 2 vs 3 on one rank (is T=2 still the right default now that the engine can
# measure the depth?): bench.py at L=512 and L=1024 fp64, each depth pinned, random init.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-f64d}
mkdir -p $O
cd $R
for L in 512 1024; do
  for f in 2 3; do
    timeout -k 10 240 python bench.py --precision Float64 --L $L --fuse $f --steps 60 --warmup 12 > $O/L${L}_f$f.json 2> $O/L${L}_f$f.err || exit 1
  done
done
echo "exit 0"
