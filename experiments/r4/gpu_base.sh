# Round 4 baseline on a fresh box: the GPU suite, the driver's N=1 and N=2 commands.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4base}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err
echo "exit $?"
