# Round 4: the one-sided 256^3 rank of the 2x2x2 grid with the folded-strip candidate (k = 2, 3).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4split2}
mkdir -p $O
cd $R
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 2 3 --out $O/onesided.json > $O/onesided.log 2>&1 &&
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 3 --out $O/allsides.json > $O/allsides.log 2>&1
echo "exit $?"
