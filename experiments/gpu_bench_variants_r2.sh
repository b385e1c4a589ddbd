# The driver's bench command three times (one process each) plus its kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-bv}
mkdir -p $O
cd $R
for i in 1 2 3; do
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
done
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1
echo "exit $?"
