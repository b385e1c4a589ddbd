# Round 3 final check on one fresh box: the whole GPU suite, the driver's N=1 command (twice), the
# driver's N=2 command self-launched on the one GPU, smoke(), a kernel trace of the N=1 command and
# SQ counters of the small-grid block kernel (L=64), each step under its own time limit.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-final3}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1b.json 2>> $O/n1.err &&
timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace512 -o run -- python bench.py --steps 20 --warmup 5 > $O/trace512.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc64 -o run -- python bench.py --L 64 --steps 400 --warmup 40 > $O/pmc64.log 2>&1
echo "exit $?"
