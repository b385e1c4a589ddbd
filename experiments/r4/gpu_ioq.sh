# Round 4: the output queue (output_queue = 1 / 2 / 3 steps in flight) on the reference's L=64
# example end to end, after the I/O GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4ioq}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_io.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for q in 1 2 3 2 1; do
  mkdir -p $O/ex64_q$q && cd $O/ex64_q$q && sed -e 's/^output = .*/output = "ex64.bp"/' $R/examples/settings-files.toml > ex.toml &&
  echo "perf_log = \"perf.jsonl\"" >> ex.toml && echo "output_queue = $q" >> ex.toml &&
  timeout -k 10 300 python3 $R/gray-scott.py ex.toml > ex.log 2> ex.err &&
  tail -n 1 perf.jsonl >> $O/summary_q$q.jsonl && rm -rf ex64.bp || exit 1
done
echo "exit $?"
