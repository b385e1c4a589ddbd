# Round 4: the watchdog wait spins (no sleep) for its first 50 ms: the IPC / RCCL GPU tests, then
# the driver's 2-rank command three times (both ranks on the one GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4wait}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_rccl_loopback.py tests/test_gpu_phases.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2954$i bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2_$i.json 2> $O/n2_$i.err || exit 1
done
echo "exit $?"
