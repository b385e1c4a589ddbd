set -e
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_rccl_loopback.py > gpurun_out/mr3.log 2>&1 || { tail -30 gpurun_out/mr3.log; exit 1; }
tail -2 gpurun_out/mr3.log
timeout -k 10 300 python scripts/bench_overlap_split.py --L 512 --nz 64 --k 3 2>/dev/null | grep "^{" | cut -c1-200
