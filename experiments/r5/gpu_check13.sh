# Round 5, lease 13: carried exchanges (the next exchange packed by the producers at the end of
# their march) -- correctness, then the cost against one-unit start-packed tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c31}
mkdir -p $O
cd $R
export TMPDIR=/tmp
export GS_COMM_TIMEOUT=60
timeout -k 10 900 python -u -m pytest tests/test_gpu_gated.py -m gpu -x -v --timeout 500 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 600 python -u scripts/bench_gated.py --n 256 --k 3 --nbrs z plus all --gate-modes 1 3 0 --gated-only --out $O/gated.json > $O/gated.log 2>&1 &&
timeout -k 10 200 python bench.py --steps 100 --warmup 20 > $O/bench.json 2> $O/bench.err
echo "exit $?"
