# Round 4: in-process A/B of the fused kernel's production candidates at L=512 T=3 from the random
# init, in the driver's window (18 timed steps after warm-up), the ablation build (which holds the
# production shapes too): Philox keys in VGPRs (-abl4) vs SALU-rebuilt keys, PF 1 vs 2, the
# 64-row tile; then a kernel trace of the driver's N=1 command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4ab}
mkdir -p $O
cd $R
export TMPDIR=/tmp
GS_HIP_VARIANT=abl timeout -k 10 600 python scripts/tune_inproc.py --L 512 --fuse 3 --init random --warmup 6 --steps 18 --rounds 5 --sched 1 2 --cfg "" 4x12:2s 4x12:1s 4x12:2s-abl4 4x12:1s-abl4 4x16:1s --out $O/ab512.json > $O/ab512.log 2>&1 &&
GS_HIP_VARIANT=abl timeout -k 10 300 python scripts/tune_inproc.py --L 256 --fuse 3 --init random --warmup 6 --steps 60 --rounds 5 --sched 1 2 --cfg "" 4x12:1s 4x12:1s-abl4 4x16:1s 4x8:1s --out $O/ab256.json > $O/ab256.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace512 -o run -- python bench.py --steps 20 --warmup 5 > $O/trace512.log 2>&1
echo "exit $?"
