set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_rccl_loopback.py > gpurun_out/kt.log 2>&1 || { tail -30 gpurun_out/kt.log; exit 1; }
tail -1 gpurun_out/kt.log
timeout -k 10 400 python scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:1s 4x12:1s-abl64 --sched 2 --rounds 6 > gpurun_out/ab_ar31v2.txt 2>&1
timeout -k 10 400 python scripts/tune_inproc.py --L 256 --fuse 2 --cfg 4x12:2s 4x12:2s-abl64 --sched 1 --rounds 6 >> gpurun_out/ab_ar31v2.txt 2>&1
grep median gpurun_out/ab_ar31v2.txt
for L in 512 256; do timeout -k 10 300 python bench.py --L $L 2>/dev/null | cut -c1-150; done
