# Round 4 final tree: rocprofv3 kernel statistics of the driver's N=1 command and of L=256.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4stats}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/l512 -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/l512.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/l256 -o run -- python3 $R/bench.py --L 256 --steps 300 --warmup 30 > $O/l256.log 2>&1
echo "exit $?"
