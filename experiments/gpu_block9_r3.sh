# Round 3: k_block with the Philox round keys in VGPRs (blk*k): bitwise tests, in-process A/B vs the
# SALU-key shapes at L=64/48, the L=64 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-blk3k}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_block.py -x -v -s --timeout 120 --timeout-method thread > $O/blocktests.log 2>&1 &&
timeout -k 10 300 python scripts/tune_inproc.py --L 64 48 --fuse 2 3 --cfg 4x6:2s blk8x2w16 blk4x4w16 blk8x2w16k blk4x4w16k --sched 2 --init random --rounds 3 --steps 400 > $O/ab.txt 2>&1 &&
timeout -k 10 120 python bench.py --L 64 --steps 2000 --warmup 200 > $O/l64.json 2> $O/l64.err &&
timeout -k 10 120 python bench.py --L 64 --steps 2000 --warmup 200 > $O/l64b.json 2> $O/l64b.err
echo "exit $?"
