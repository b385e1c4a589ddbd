# Overlap split costs with the current kernel (autotuned launches) for the strong-scaling model, and
# the RCCL-loopback wall time per pass of the chained vs the sequential z-slab / packed passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-split}
mkdir -p $O
cd $R
timeout -k 10 300 python scripts/bench_overlap_split.py --nz 64 128 256 --k 3 > $O/split_z.txt 2>&1 &&
timeout -k 10 200 python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 2 3 > $O/split_p.txt 2>&1 &&
timeout -k 10 200 python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 2 3 > $O/split_p1.txt 2>&1 &&
for m in zplanes packed; do
  if [ $m = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
  timeout -k 10 100 python scripts/trace_overlap.py --mode $m $A --fuse 3 --passes 60 --overlap off >> $O/wall.txt 2>&1 &&
  timeout -k 10 100 python scripts/trace_overlap.py --mode $m $A --fuse 3 --passes 60 >> $O/wall.txt 2>&1 || exit 1
done
echo "exit $?"
