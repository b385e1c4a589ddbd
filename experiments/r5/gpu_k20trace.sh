# Round 5: kernel timeline of the driver's bench command (K=20, W=5): per-dispatch start / end.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5k20}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o k20 -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "exit $?"
