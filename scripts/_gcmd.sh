set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_multirank.py -k bench_two_ranks > gpurun_out/t_bench2.log 2>&1 || { tail -30 gpurun_out/t_bench2.log; exit 1; }
tail -2 gpurun_out/t_bench2.log
timeout -k 10 300 python bench.py --L 1024 --steps 60 --warmup 6 > gpurun_out/b1024f32.json 2>/dev/null
timeout -k 10 300 python bench.py --L 1024 --precision Float64 --steps 40 --warmup 4 > gpurun_out/b1024f64.json 2>/dev/null
timeout -k 10 300 python bench.py --L 512 --precision Float64 --steps 100 --warmup 10 > gpurun_out/b512f64.json 2>/dev/null
for f in b1024f32 b1024f64 b512f64; do python -c "import json; d=json.load(open('gpurun_out/$f.json')); print('$f', d['value'], d['ms_per_step'], d['config']['fuse_steps'], d['config']['fused_kernel'])"; done
