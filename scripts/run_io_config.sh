#!/bin/bash
# I/O-inclusive run of the L=512 checkpoint config on one GPU, then a restart from the last
# checkpoint; writes the timing summary (perf log) under gpurun_out/.
set -e
out=${1:-gpurun_out/io512}
mkdir -p "$out"
cd "$out"
cfg=$GRAFT_REPO_ROOT/examples/l512-checkpoint.toml
[ -z "$GRAFT_REPO_ROOT" ] && cfg=../../examples/l512-checkpoint.toml
sed -e 's/^steps = .*/steps = 400/' "$cfg" > run.toml
timeout -k 10 600 python3 "${GRAFT_REPO_ROOT:-../..}/gray-scott.py" run.toml > run.log 2>&1
sed -e 's/^steps = .*/steps = 600/' -e 's/^restart = .*/restart = true/' -e 's/^perf_log = .*/perf_log = "perf-restart.jsonl"/' -e 's/^output = .*/output = "gs-restart.bp"/' run.toml > restart.toml
timeout -k 10 600 python3 "${GRAFT_REPO_ROOT:-../..}/gray-scott.py" restart.toml > restart.log 2>&1
rm -rf gs-512L-F32.bp ckpt-512L-F32.bp gs-restart.bp ckpt-512L-F32.bp.old
tail -n 1 perf-512L.jsonl > summary.json
tail -n 1 perf-restart.jsonl > summary_restart.json
echo done
