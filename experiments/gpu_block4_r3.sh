# Round 3: block kernel v2 (Philox in the load shadow, 16-wave variants): bitwise tests, small-grid
# benches, in-process A/B, an L=64 kernel trace (csv), then the whole GPU suite, the driver's N=1
# bench command and smoke().
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-blk3d}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -v -s --timeout 120 --timeout-method thread > $O/blocktests.log 2>&1 &&
timeout -k 10 120 python bench.py --L 64 --steps 2000 --warmup 200 > $O/l64.json 2> $O/l64.err &&
timeout -k 10 120 python bench.py --L 64 --steps 2000 --warmup 200 > $O/l64b.json 2> $O/l64b.err &&
timeout -k 10 300 python scripts/tune_inproc.py --L 64 48 32 --fuse 2 3 --cfg 4x6:2s blk8x2w8 blk4x4w8 blk8x2w16 blk4x4w16 blk8x4w16 --sched 2 --init random --rounds 3 --steps 400 > $O/ab.txt 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof64 -o run -- python bench.py --L 64 --steps 400 --warmup 40 > $O/prof64.log 2>&1 &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo "exit $?"
