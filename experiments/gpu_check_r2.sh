# GPU check used this round: correctness of the production kernels first, then the driver's
# bench command (twice), a long bench, and a kernel trace of the driver command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-chk}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > $O/gputest_kernels.log 2>&1 &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver2.json 2>> $O/bench_driver.err &&
timeout -k 10 150 python bench.py --gpus 1 --steps 400 --warmup 40 > $O/bench_long.json 2> $O/bench_long.err &&
timeout -k 10 150 python scripts/power_probe.py --passes 40 > $O/probe.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_driver.log 2>&1
echo "exit $?"
