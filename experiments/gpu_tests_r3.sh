# Round 3: the whole GPU suite (one process, per-test time limits), then the driver's bench
# commands at N=1 and N=2 (self-launched on the one GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-t3}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err
echo "exit $?"
