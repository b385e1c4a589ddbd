# Round 3: IPC tests (the pack's store-ack wait replacing the per-wave system fence), then the
# emulated-exchange overlap comparison (experiments/gpu_emulate_r3.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-emu3b}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipc.py -x -v --timeout 300 --timeout-method thread > $O/ipc_tests.log 2>&1 &&
GS_OUT=${GS_OUT:-emu3b} bash experiments/gpu_emulate_r3.sh
