set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof64 -o run -- python3 bench.py --L 64 --steps 200 --warmup 20 > gpurun_out/prof64.log 2>&1
find gpurun_out/prof64 -type f | head
