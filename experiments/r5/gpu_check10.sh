# Round 5, lease 10: the example's output step after the native writer thread and the warmed ring.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c23}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_io.py tests/test_functional.py tests/test_simulation.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python scripts/profile_output.py --repeat 4 > $O/output_prof.log 2>&1 &&
for i in 1 2 3; do timeout -k 10 120 python gray-scott.py examples/settings-files.toml >> $O/example.log 2>&1 || exit 1; done
echo "exit $?"
