set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py > gpurun_out/kt.log 2>&1 || { tail -30 gpurun_out/kt.log; exit 1; }
tail -1 gpurun_out/kt.log
for L in 512 1024; do timeout -k 10 300 python bench.py --L $L --precision Float64 --steps 60 --warmup 6 2>/dev/null | cut -c1-160; done
