# Pack / unpack kernels sized by the messages' cells: packed-plan GPU tests, then the packed-rank loopback
# timeline (pack / RCCL / unpack durations) and wall time per pass.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-pack}
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_gpu_rccl_loopback.py tests/test_gpu_multirank.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread > $O/gputest.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 100 python scripts/trace_overlap.py --mode packed --L 256 --nz 256 --fuse 3 --passes 60 --overlap off >> $O/wall.txt 2>&1 &&
timeout -k 10 100 python scripts/trace_overlap.py --mode packed --L 256 --nz 256 --fuse 3 --passes 60 >> $O/wall.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_p -o run -- python3 $R/scripts/trace_overlap.py --mode packed --L 256 --nz 256 > $O/tr_p.log 2>&1 &&
GS_OVERLAP_CHAIN=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_p_off -o run -- python3 $R/scripts/trace_overlap.py --mode packed --L 256 --nz 256 --overlap off > $O/tr_p_off.log 2>&1
echo "exit $?"
