# Pipeline-fill level skip: correctness (kernel / headline / loopback GPU tests, exactness of the
# -abl16 variant that computes every level), in-process A/B (production vs -abl16, random state),
# overlap split costs with and without the skip, and the driver's bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-fill}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_headline.py tests/test_gpu_rccl_loopback.py -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "tests failed"; exit 1; }
GS_HIP_VARIANT=abl timeout -k 10 200 python scripts/abl_digest.py --cfg 4x12:1s 4x12:1s-abl16 4x8:1s 4x8:1s-abl16 > $O/digest.txt 2>&1 &&
GS_HIP_VARIANT=abl timeout -k 10 400 python scripts/tune_inproc.py --L 512 256 128 --fuse 3 --cfg 4x12:1s 4x12:1s-abl16 4x8:1s 4x8:1s-abl16 --sched 1 2 --init random --rounds 3 > $O/ab.txt 2>&1 &&
GS_HIP_VARIANT=abl GS_FUSED_CFG=4x12:1s timeout -k 10 200 python scripts/bench_overlap_split.py --nz 64 --k 3 > $O/split_skip.txt 2>&1 &&
GS_HIP_VARIANT=abl GS_FUSED_CFG=4x12:1s-abl16 timeout -k 10 200 python scripts/bench_overlap_split.py --nz 64 --k 3 > $O/split_noskip.txt 2>&1 &&
GS_HIP_VARIANT=abl GS_FUSED_CFG=4x8:1s timeout -k 10 200 python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 3 >> $O/split_skip.txt 2>&1 &&
GS_HIP_VARIANT=abl GS_FUSED_CFG=4x8:1s-abl16 timeout -k 10 200 python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 3 >> $O/split_noskip.txt 2>&1 &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver2.json 2>> $O/bench_driver.err &&
timeout -k 10 150 python bench.py --gpus 1 --steps 400 --warmup 40 > $O/bench_long.json 2> $O/bench_long.err
echo "exit $?"
