# Round 5, lease 4: the output step with the snapshot kernel's min / max (tests + the example's
# host-side breakdown, scripts/profile_output.py) and the example end to end.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c4}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_io.py -m gpu -k "snapshot or async or gpu" -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python scripts/profile_output.py --repeat 4 > $O/output_prof.log 2>&1 &&
timeout -k 10 300 python gray-scott.py examples/settings-files.toml > $O/example.log 2>&1
echo "exit $?"
