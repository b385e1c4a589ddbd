# Round 5, lease 14: in-march carry for z slabs (a carried pass's send planes stored into the
# peers' landing slot from inside the march) -- correctness, then the z-slab cost.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c33}
mkdir -p $O
cd $R
export TMPDIR=/tmp
export GS_COMM_TIMEOUT=60
timeout -k 10 900 python -u -m pytest tests/test_gpu_gated.py -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 600 python -u scripts/bench_gated.py --n 256 --k 3 --nbrs z --emulate-us 0 30 --gate-modes 1 3 0 --gated-only --out $O/gated.json > $O/gated.log 2>&1
echo "exit $?"
