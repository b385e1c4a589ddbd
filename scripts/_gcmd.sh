set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_rccl_loopback.py > gpurun_out/mr5.log 2>&1 || { tail -30 gpurun_out/mr5.log; exit 1; }
tail -2 gpurun_out/mr5.log
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 2 3 2>/dev/null | grep "^{" | cut -c1-200
