# Round 5 final check: full GPU suite, the driver's bench (twice) and the default one, a
# kernel-trace profile of the bench, and the gated table kinds on the 256^3 loopback rank.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5f3}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver2.json 2> $O/bench_driver2.err &&
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench -- python3 bench.py --steps 100 --warmup 10 > $O/prof.log 2>&1 &&
timeout -k 10 600 python -u scripts/bench_gated.py --n 256 --k 3 --nbrs z plus all --gate-modes 1 3 0 --gated-only --out $O/gated.json > $O/gated.log 2>&1
echo "exit $?"
