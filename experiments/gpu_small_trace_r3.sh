# Round 3: where an L=64 pass's time goes (kernel durations vs gaps between launches).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-small3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/bench.py --L 64 --steps 2000 --warmup 200 > $O/l64.json 2> $O/l64.err &&
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --L 64 --steps 400 --warmup 40 --check none > $O/trace.log 2>&1
echo "exit $?"
