# Round 4 check on one fresh box: the whole GPU suite, the driver's N=1 command (twice), the
# reference example size (L=64), the driver's N=2 command self-launched on the one GPU, smoke(),
# a kernel trace of the N=1 command, each step under its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4full}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1b.json 2>> $O/n1.err &&
timeout -k 10 200 python bench.py --L 64 --steps 2000 --warmup 200 > $O/n1_L64.json 2> $O/n1_L64.err &&
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace512 -o run -- python bench.py --steps 20 --warmup 5 > $O/trace512.log 2>&1
echo "exit $?"
