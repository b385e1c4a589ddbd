# Final round check: the whole GPU test suite, smoke(), the driver's bench command (twice), and the driver's
# multi-rank invocation (torchrun, 2 ranks) rehearsed on ONE GPU (RCCL refuses two ranks per device: the
# data-path tuning falls back to the host transport).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-final}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || { echo "gpu tests failed"; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver2.json 2>> $O/bench_driver.err &&
GS_COMM_TIMEOUT=60 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 20 --warmup 5 > $O/r2_torchrun.json 2> $O/r2_torchrun.err
echo "exit $?"
