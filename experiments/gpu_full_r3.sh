# Round 3: the whole GPU suite, the driver's bench command at N=1 (twice), a long N=1 run, and
# the 8-rank fp64 check of the timed path on one GPU.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-full3}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1b.json 2>> $O/n1.err &&
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > $O/n1_long.json 2> $O/n1_long.err
echo "exit $?"
