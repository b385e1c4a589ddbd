# Round 4: (1) shell changes (x/y-only k_slab <= 256 VGPRs; variant 2 = z slabs beside the x/y
# slabs on a side stream) + padded-row boundary fill + the SALU-lean block kernel (k_block_sl):
# correctness tests, the 256^3 shell splits, L=64 block A/B and bench, the driver's N=1 command;
# (2) the fused-kernel A/B (experiments/r4/gpu_ab.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4shell}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_block.py tests/test_gpu_overlap_shell.py tests/test_gpu_kernels.py tests/test_gpu_multirank.py tests/test_gpu_oracle.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python scripts/tune_inproc.py --L 64 --fuse 2 3 --init random --warmup 30 --steps 600 --rounds 3 --sched 0 --cfg blk8x2w16 blk8x2w16s blk4x4w16 blk4x4w16s blk8x2w8 blk8x2w8s --out $O/ab64.json > $O/ab64.log 2>&1 &&
timeout -k 10 200 python bench.py --L 64 --steps 2000 --warmup 200 > $O/n1_L64.json 2> $O/n1_L64.err &&
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 3 2 --out $O/split_onesided.json > $O/split.log 2>&1 &&
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 3 --out $O/split_allsides.json >> $O/split.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
GS_OUT=r4ab bash experiments/r4/gpu_ab.sh
echo "exit $?"
