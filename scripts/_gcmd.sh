set -e
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 2 3 --out gpurun_out/split_packed.json > gpurun_out/split_packed.log 2>&1
timeout -k 10 300 python scripts/bench_overlap_split.py --L 512 --nz 64 128 --k 2 3 --out gpurun_out/split_z.json > gpurun_out/split_z.log 2>&1
cat gpurun_out/split_packed.log gpurun_out/split_z.log | grep "^{"
