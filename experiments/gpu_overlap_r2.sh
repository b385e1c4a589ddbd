# Overlap schedules on ONE GPU through the RCCL loopback: correctness (loopback / multi-rank GPU
# tests), split costs, wall time per pass (overlap off, chained, one pass at a time), timelines.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-ovl}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl_loopback.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread > $O/gputest_ovl.log 2>&1 || { echo "tests failed"; exit 1; }
[ -n "$GS_SPLIT" ] && { timeout -k 10 200 python scripts/bench_overlap_split.py --nz 64 --k 3 > $O/split_z.txt 2>&1 &&
timeout -k 10 200 python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 2 3 > $O/split_p.txt 2>&1 &&
timeout -k 10 200 python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 2 3 > $O/split_p1.txt 2>&1 || { echo "split failed"; exit 1; }; }
for m in zplanes packed; do
  if [ $m = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
  for f in 3 2; do
    timeout -k 10 100 python scripts/trace_overlap.py --mode $m $A --fuse $f --passes 60 --overlap off >> $O/wall.txt 2>&1 &&
    timeout -k 10 100 python scripts/trace_overlap.py --mode $m $A --fuse $f --passes 60 >> $O/wall.txt 2>&1 &&
    GS_OVERLAP_CHAIN=0 timeout -k 10 100 python scripts/trace_overlap.py --mode $m $A --fuse $f --passes 60 >> $O/wall.txt 2>&1 &&
    true || { echo "wall $m $f failed"; exit 1; }
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_z -o run -- python3 $R/scripts/trace_overlap.py --mode zplanes --L 512 --nz 64 > $O/tr_z.log 2>&1 &&
GS_OVERLAP_CHAIN=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_z1 -o run -- python3 $R/scripts/trace_overlap.py --mode zplanes --L 512 --nz 64 > $O/tr_z1.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_p -o run -- python3 $R/scripts/trace_overlap.py --mode packed --L 256 --nz 256 > $O/tr_p.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_p2 -o run -- python3 $R/scripts/trace_overlap.py --mode packed --L 256 --nz 256 --fuse 2 > $O/tr_p2.log 2>&1
echo "exit $?"
