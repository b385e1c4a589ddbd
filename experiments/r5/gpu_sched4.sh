# Round 5: work schedule 4 (equal shares of the z-block-major plane order) -- bitwise vs sched 2,
# then in-process A/B against schedules 1 / 2 at L=512 / 256, T=3 / 2, and the driver's bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5s4}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_oracle.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 600 python -u scripts/tune_inproc.py --L 512 256 --fuse 3 2 --cfg 4x12:1s 4x12:1sf --sched 1 2 4 --rounds 3 --init random --out $O/tune.json > $O/tune.log 2>&1 &&
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver2.json 2> $O/bench_driver2.err &&
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err
echo "exit $?"
