# Round 5: 4x12:3s with the step-uniform Philox words in VGPRs (ablation entry 56) against the
# production 4x12:1s at L=512 / 1024 T=3, 5 interleaved rounds, random and seed init.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5pf3}
mkdir -p $O
cd $R
export TMPDIR=/tmp
export GS_HIP_VARIANT=abl
timeout -k 10 600 python -u scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:1s 4x12:3s-abl128 --sched 1 2 --rounds 5 --init random --out $O/r512.json > $O/r512.log 2>&1 &&
timeout -k 10 600 python -u scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:1s 4x12:3s-abl128 --sched 2 --rounds 5 --steps 240 --out $O/s512.json > $O/s512.log 2>&1 &&
timeout -k 10 600 python -u scripts/tune_inproc.py --L 1024 --fuse 3 --cfg 4x12:1s 4x12:3s-abl128 --sched 2 --rounds 3 --steps 30 --init random --out $O/r1024.json > $O/r1024.log 2>&1
echo "exit $?"
