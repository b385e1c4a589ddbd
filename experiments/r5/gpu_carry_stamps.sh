# Round 5: where a carried exchange's time goes (gate_stamps incl. the producers' carry)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5cs}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/bench_gated.py --n 256 --k 3 --nbrs z plus all --emulate-us 0 --gate-modes 1 3 --gated-only --stamps --out $O/gated.json > $O/gated.log 2>&1
echo "exit $?"
