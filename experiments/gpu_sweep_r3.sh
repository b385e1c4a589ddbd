# Round 3 final sweep on one fresh box: bench.py per size / precision with the final code (autotuned
# tile, measured depth on one rank), every row golden-checked after timing; then the driver's N=4 and N=8
# commands self-launched with all ranks on the one GPU (tuning wall time and the table, not scaling).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-sweep3}
mkdir -p $O
cd $R
run() { # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; return 1; }
}
run l128 150 --L 128 --steps 1000 --warmup 100 &&
run l192 150 --L 192 --steps 1000 --warmup 100 &&
run l256 150 --L 256 --steps 1000 --warmup 100 &&
run l512 200 --L 512 --steps 400 --warmup 40 &&
run l1024 300 --L 1024 --steps 60 --warmup 6 &&
run l512f64 200 --L 512 --precision Float64 --steps 200 --warmup 20 &&
run l1024f64 300 --L 1024 --precision Float64 --steps 30 --warmup 6 &&
run n4 300 --gpus 4 --steps 20 --warmup 5 &&
run n8 400 --gpus 8 --steps 20 --warmup 5
echo "exit $?"
