# Round 3: the I/O-inclusive configs with the final code: BASELINE config 5 on one GPU (L=512 fp32,
# output + checkpoint every 100 steps, 400 steps, then a restart run) and the reference's example
# config (L=64, 1000 steps, output every 10 steps) end to end.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-io3}
mkdir -p $O/ex64
cd $R
true &&
cd $O/ex64 && sed -e 's/^output = .*/output = "ex64.bp"/' $R/examples/settings-files.toml > ex.toml &&
echo 'perf_log = "perf-ex64.jsonl"' >> ex.toml &&
timeout -k 10 300 python3 $R/gray-scott.py ex.toml > ex.log 2> ex.err &&
tail -n 1 perf-ex64.jsonl > summary.json && rm -rf ex64.bp
echo "exit $?"
