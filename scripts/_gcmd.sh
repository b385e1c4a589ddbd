set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_rccl_loopback.py > gpurun_out/lb.log 2>&1 || { tail -30 gpurun_out/lb.log; exit 1; }
tail -1 gpurun_out/lb.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/ovl_p gpurun_out/ovl_p0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovl_p -o run -- python3 scripts/trace_overlap.py --mode packed --L 256 --nz 256 --fuse 2 > gpurun_out/ovl_p.log 2>&1
GS_OVERLAP_CHAIN=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ovl_p0 -o run -- python3 scripts/trace_overlap.py --mode packed --L 256 --nz 256 --fuse 2 > gpurun_out/ovl_p0.log 2>&1
python3 scripts/trace_overlap.py --summarise gpurun_out/ovl_p > gpurun_out/ovl_p.txt
python3 scripts/trace_overlap.py --summarise gpurun_out/ovl_p0 > gpurun_out/ovl_p0.txt
tail -12 gpurun_out/ovl_p.txt; tail -8 gpurun_out/ovl_p0.txt
