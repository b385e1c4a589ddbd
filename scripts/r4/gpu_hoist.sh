# Round 4: A/B of the Philox blocks drawn before the workgroup barrier (-abl512 all levels,
# -abl1024 top level, -abl1536 top two) against the production 4x12:1s, L=512 / L=256 T=3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4hoist}
mkdir -p $O
cd $R
GS_HIP_VARIANT=abl timeout -k 10 600 python scripts/tune_inproc.py --L 512 --fuse 3 --init random --warmup 6 --steps 18 --rounds 5 --sched 1 2 --cfg 4x12:1s 4x12:1s-abl512 4x12:1s-abl1024 4x12:1s-abl1536 --out $O/ab512.json > $O/ab512.log 2>&1 &&
GS_HIP_VARIANT=abl timeout -k 10 600 python scripts/tune_inproc.py --L 256 --fuse 3 --init random --warmup 10 --steps 60 --rounds 5 --sched 1 2 --cfg 4x12:1s 4x12:1s-abl512 4x12:1s-abl1024 4x12:1s-abl1536 --out $O/ab256.json > $O/ab256.log 2>&1
echo "exit $?"
