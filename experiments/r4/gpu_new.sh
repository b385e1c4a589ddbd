# Round 4: the new / changed GPU tests (oracle, phases, IPC system stores, debug switches,
# untuned depth), then the driver's N=1 command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4new}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_oracle.py tests/test_gpu_phases.py tests/test_gpu_ipc.py tests/test_gpu_block.py tests/test_gpu_rccl_loopback.py tests/test_gpu_headline.py -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err
echo "exit $?"
