# Round check: the whole GPU test suite, smoke(), the driver's bench command, BASELINE configs on one GPU
# (L=256 1000 steps, L=1024 fp64), and the 8-rank self-launched bench rehearsal on one GPU (host transport).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-round}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 200 python bench.py --gpus 1 --L 256 --steps 1000 --warmup 60 > $O/bench_L256.json 2> $O/bench_L256.err &&
timeout -k 10 300 python bench.py --gpus 1 --L 1024 --precision Float64 --steps 30 --warmup 4 > $O/bench_L1024_f64.json 2> $O/bench_L1024_f64.err &&
timeout -k 10 420 python bench.py --gpus 8 --steps 20 --warmup 5 --transport host > $O/r8_host.json 2> $O/r8_host.err
echo "exit $?"
