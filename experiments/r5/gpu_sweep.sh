# Round 5 final sweep on one fresh box: the driver's N=1 command three times, then bench.py per
# size / precision with the final code, every row golden-checked after timing; then the
# reference's example config (L=64, output every 10 steps) end to end.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5sweep}
mkdir -p $O
cd $R
run() { # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/$n.json 2> $O/$n.err || { echo "bench $n failed"; return 1; }
}
run drv1 200 --gpus 1 --steps 20 --warmup 5 &&
run drv2 200 --gpus 1 --steps 20 --warmup 5 &&
run drv3 200 --gpus 1 --steps 20 --warmup 5 &&
run l512 200 --L 512 --steps 400 --warmup 40 &&
run l1024 300 --L 1024 --steps 60 --warmup 6 &&
run l256 150 --L 256 --steps 1000 --warmup 100 &&
run l128 150 --L 128 --steps 1000 --warmup 100 &&
run l64 150 --L 64 --steps 2000 --warmup 200 &&
run l512f64 200 --L 512 --precision Float64 --steps 200 --warmup 20 &&
run l1024f64 300 --L 1024 --precision Float64 --steps 30 --warmup 6 &&
mkdir -p $O/ex64 && cd $O/ex64 && sed -e 's/^output = .*/output = "ex64.bp"/' $R/examples/settings-files.toml > ex.toml &&
echo 'perf_log = "perf-ex64.jsonl"' >> ex.toml &&
timeout -k 10 300 python3 $R/gray-scott.py ex.toml > ex.log 2> ex.err &&
tail -n 1 perf-ex64.jsonl > summary.json && rm -rf ex64.bp
echo "exit $?"
# one-GPU rehearsals of the multi-rank bench (ranks share the card: data-path checks, not scaling)
cd $R
timeout -k 10 400 python bench.py --gpus 2 --L 256 --steps 60 --warmup 10 --timeout 360 > $O/n2.json 2> $O/n2.err &&
timeout -k 10 500 python bench.py --gpus 4 --L 256 --steps 60 --warmup 10 --timeout 460 > $O/n4.json 2> $O/n4.err
echo "rehearsal exit $?"
