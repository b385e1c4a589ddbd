# Round 3: the cell-granular overlap -- the shell kernel's bit-exactness (inner + shell == full
# pass), the multi-rank overlapped paths, then the split costs for the headline sub-domains.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-sh3}
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_overlap_shell.py -x -v --timeout 120 --timeout-method thread > $O/shell_tests.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_ipc.py tests/test_gpu_rccl_loopback.py -x -v --timeout 300 --timeout-method thread > $O/mr_tests.log 2>&1 &&
timeout -k 10 200 python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 3 2 > $O/split_onesided.txt 2>&1 &&
timeout -k 10 200 python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 3 > $O/split_packed.txt 2>&1 &&
timeout -k 10 200 python scripts/bench_overlap_split.py --nz 64 128 --k 3 > $O/split_zslab.txt 2>&1
echo "exit $?"
