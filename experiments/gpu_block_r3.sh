# Round 3: the small-grid block kernel (csrc/hip/block.hpp): bitwise tests, the L=64 bench
# (autotuner sees the blk* candidates), in-process A/B of every candidate at small L, then the
# whole GPU suite and the driver's N=1 bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-blk3}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -v -s --timeout 120 --timeout-method thread > $O/blocktests.log 2>&1 &&
timeout -k 10 120 python bench.py --L 64 --steps 2000 --warmup 200 > $O/l64.json 2> $O/l64.err &&
timeout -k 10 300 python scripts/tune_inproc.py --L 64 48 32 --fuse 2 3 --cfg 4x6:2s 4x8:1s blk8x2w8 blk4x2w4 blk8x1w8 blk4x4w8 blk4x1w4 --sched 2 --init random --rounds 3 --steps 400 > $O/ab.txt 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "exit $?"
