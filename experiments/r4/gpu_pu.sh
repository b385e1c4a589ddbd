# Round 4: PU (step-uniform Philox words in VGPRs) default on the 1-prefetch KV shapes:
# GPU suite, A/B against the PU-off ablation, N=1 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4pu}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 &&
GS_HIP_VARIANT=abl timeout -k 10 600 python scripts/tune_inproc.py --L 512 --fuse 3 --init random --warmup 6 --steps 18 --rounds 5 --sched 1 2 --cfg 4x12:1s 4x12:1s-abl256 4x12:2s --out $O/ab512.json > $O/ab512.log 2>&1 &&
timeout -k 10 400 python bench.py > $O/n1.json 2> $O/n1.err &&
timeout -k 10 400 python bench.py > $O/n1b.json 2> $O/n1b.err
echo "exit $?"
