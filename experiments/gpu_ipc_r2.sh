# IPC peer-write transport on one MI355X: loopback + multi-process tests, then the pack / chain
# regressions (RCCL loopback, multi-rank host transport) and the driver's bench command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-ipc1}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipc.py -x -v --timeout 120 --timeout-method thread > $O/ipc.log 2>&1 || { echo "ipc tests failed"; tail -30 $O/ipc.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl_loopback.py tests/test_gpu_multirank.py -x -q --timeout 120 --timeout-method thread > $O/regress.log 2>&1 || { echo "regression tests failed"; tail -30 $O/regress.log; exit 1; }
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err
echo "exit $?"
tail -n 3 $O/ipc.log $O/regress.log
