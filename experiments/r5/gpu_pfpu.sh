# Round 5: 2- and 3-plane prefetch with the step-uniform Philox words in VGPRs (ablation build,
# entries 55 / 56) against the production 4x12:1s, in-process A/B at L=512, T=2 / T=3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5pf}
mkdir -p $O
cd $R
export TMPDIR=/tmp
export GS_HIP_VARIANT=abl
timeout -k 10 900 python -u scripts/tune_inproc.py --L 512 --fuse 2 3 --cfg 4x12:1s 4x12:2s 4x12:2s-abl128 4x12:3s-abl128 --sched 1 2 --rounds 3 --init random --out $O/tune.json > $O/tune.log 2>&1
echo "exit $?"
