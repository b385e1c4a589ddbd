# Round 4: A/B of the step-uniform Philox words in VGPRs (-abl128) against the production shapes
# (Philox keys in VGPRs now default: 4x12:1s / 4x12:2s; -abl64 = keys on the SALU), L=512 T=3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4ab2}
mkdir -p $O
cd $R
GS_HIP_VARIANT=abl timeout -k 10 600 python scripts/tune_inproc.py --L 512 --fuse 3 --init random --warmup 6 --steps 18 --rounds 5 --sched 1 2 --cfg 4x12:1s 4x12:1s-abl256 4x12:2s 4x12:1s-abl64 --out $O/ab512.json > $O/ab512.log 2>&1
echo "exit $?"
