# Kernel-variant check: correctness of the production kernels, then in-process A/B of tiles /
# schedules on the benchmark's random state (power-limited) and on the seed state, then the
# driver's bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-tune}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/gputest_kernels.log 2>&1 &&
timeout -k 10 300 python scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:2s 4x12:1s 4x16:1s 4x8:1s --sched 1 2 --init random --steps 20 --warmup 5 --rounds 3 --out $O/tune_random.json > $O/tune_random.txt 2>&1 &&
timeout -k 10 300 python scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:2s 4x12:1s 4x16:1s --sched 1 2 --steps 120 --rounds 3 --out $O/tune_seed.json > $O/tune_seed.txt 2>&1 &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 150 python bench.py --gpus 1 --steps 400 --warmup 40 > $O/bench_long.json 2> $O/bench_long.err
echo "exit $?"
