# Round 5, lease 11: gated passes with the unpack table built during the wait.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c24}
mkdir -p $O
cd $R
export TMPDIR=/tmp
export GS_COMM_TIMEOUT=60
timeout -k 10 600 python -u -m pytest tests/test_gpu_gated.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 500 python -u scripts/bench_gated.py --n 256 --k 3 --out $O/gated.json > $O/gated.log 2>&1 &&
timeout -k 10 300 python -u scripts/bench_gated.py --n 256 --k 3 --emulate-us 0 --stamps > $O/stamps.log 2>&1
echo "exit $?"
