# Round 4 (final kernel): per-rank kernel costs of the overlap split for the N = 2 / 4 / 8 sub-domains
# at L=512 (z slabs) and the one-sided 256^3 rank of the 2x2x2 grid, k = 2 and 3, no communication.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4split}
mkdir -p $O
cd $R
timeout -k 10 400 python scripts/bench_overlap_split.py --nz 64 128 256 --k 2 3 --out $O/zslab.json > $O/zslab.log 2>&1 &&
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 2 3 --out $O/onesided.json > $O/onesided.log 2>&1
echo "exit $?"
