# The reference example end to end, five fresh processes (output phase per run from the perf log).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5ex}
mkdir -p $O/ex64 && cd $O/ex64
sed -e 's/^output = .*/output = "ex64.bp"/' $R/examples/settings-files.toml > ex.toml
echo 'perf_log = "perf-ex64.jsonl"' >> ex.toml
for i in 1 2 3 4 5; do
  timeout -k 10 120 python3 $R/gray-scott.py ex.toml > ex.log 2> ex.err || exit 1
  tail -n 1 perf-ex64.jsonl >> summaries.jsonl
  rm -rf ex64.bp perf-ex64.jsonl
done
cd $R && timeout -k 10 200 python scripts/profile_output.py --repeat 3 > $O/output_prof.log 2>&1
echo "exit $?"
