# Round 3: block kernel with VGPR Philox keys: tests, L=64 bench, the whole GPU suite,
# benches, in-process A/B, an L=64 kernel trace (csv), then the whole GPU suite, the driver's N=1
# bench command and smoke().
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-blk3n}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -v -s --timeout 120 --timeout-method thread > $O/blocktests.log 2>&1 &&
timeout -k 10 120 python bench.py --L 64 --steps 2000 --warmup 200 > $O/l64.json 2> $O/l64.err &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "exit $?"
