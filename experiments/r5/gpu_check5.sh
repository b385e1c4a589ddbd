# Round 5, lease 5: gated passes (gate.hpp) -- correctness on one GPU (IPC loopback + several
# processes), the cost against the full pass (scripts/bench_gated.py), and the headline bench
# unchanged (the gated entry is its own kernel).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c5}
mkdir -p $O
cd $R
export TMPDIR=/tmp
export GS_COMM_TIMEOUT=60
timeout -k 10 900 python -u -m pytest tests/test_gpu_gated.py tests/test_gpu_ipc.py -m gpu -x -v --timeout 240 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 400 python -u scripts/bench_gated.py --n 256 --k 3 2 --out $O/gated.json > $O/gated.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > $O/bench.log 2>&1
echo "exit $?"
