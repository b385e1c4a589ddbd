# Round 5, lease 8: the output step with the native snapshot call; host write throughput of the
# box's filesystems (experiments/r5/write_probe.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c11}
mkdir -p $O
cd $R
export TMPDIR=/tmp

timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_io.py tests/test_functional.py tests/test_simulation.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python scripts/profile_output.py --repeat 4 > $O/output_prof.log 2>&1
echo "exit $?"
