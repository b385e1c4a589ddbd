set -e
mkdir -p gpurun_out
timeout -k 10 400 python scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:1s 4x16:1s 4x14:1s 4x16:2s --sched 1 2 --rounds 4 > gpurun_out/tune_tall.txt 2>&1
timeout -k 10 300 python scripts/tune_inproc.py --L 256 --fuse 2 3 --cfg 4x12:2s 4x16:1s 4x14:1s 4x16:2s --sched 1 2 --rounds 4 >> gpurun_out/tune_tall.txt 2>&1
grep median gpurun_out/tune_tall.txt
