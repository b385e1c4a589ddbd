set -e
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_gpu_multirank.py tests/test_gpu_rccl_loopback.py > gpurun_out/mr2.log 2>&1 || { tail -30 gpurun_out/mr2.log; exit 1; }
tail -2 gpurun_out/mr2.log
