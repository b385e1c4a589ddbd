# Schedule 3 check: kernel tests, in-process A/B of schedules on the random and seed states,
# the driver's bench command, and the overlap split costs with the current kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-s3}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/gputest_kernels.log 2>&1 &&
timeout -k 10 300 python scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:1s 4x12:2s --sched 1 2 3 --init random --steps 20 --warmup 5 --rounds 3 --out $O/tune_random.json > $O/tune_random.txt 2>&1 &&
timeout -k 10 300 python scripts/tune_inproc.py --L 512 1024 --fuse 3 --cfg 4x12:1s --sched 1 2 3 --steps 60 --rounds 3 --out $O/tune_seed.json > $O/tune_seed.txt 2>&1 &&
timeout -k 10 300 python scripts/tune_inproc.py --L 256 --fuse 3 --cfg 4x12:1s 4x8:1s --sched 1 2 3 --steps 200 --rounds 3 --out $O/tune_seed256.json > $O/tune_seed256.txt 2>&1 &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver2.json 2>> $O/bench_driver.err &&
timeout -k 10 300 python scripts/bench_overlap_split.py --nz 64 128 256 --k 2 3 --out $O/split_z.json > $O/split_z.txt 2>&1 &&
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 2 3 --out $O/split_p.json > $O/split_p.txt 2>&1
echo "exit $?"
