set -e
mkdir -p gpurun_out
timeout -k 10 400 python scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:1s 4x12:1s-abl32 4x12:1s-abl16 --sched 2 --rounds 6 > gpurun_out/ab_rsrc.txt 2>&1
timeout -k 10 400 python scripts/tune_inproc.py --L 256 --fuse 2 --cfg 4x12:2s 4x12:2s-abl16 --sched 1 --rounds 6 >> gpurun_out/ab_rsrc.txt 2>&1
grep -E "median|passed|failed" gpurun_out/ab_rsrc.txt
