# Round 4: the reference's L=64 example under cProfile (main thread): where the output step's
# main-thread time goes with two output steps in flight.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4exprof}
mkdir -p $O/ex64 && cd $O/ex64
sed -e 's/^output = .*/output = "ex64.bp"/' $R/examples/settings-files.toml > ex.toml &&
echo 'perf_log = "perf.jsonl"' >> ex.toml &&
timeout -k 10 300 python3 -m cProfile -o prof.out $R/gray-scott.py ex.toml > ex.log 2> ex.err &&
python3 -c "
import pstats
p = pstats.Stats('prof.out')
p.sort_stats('cumulative').print_stats('output.py|grayscott.py|bp4.py|dist.py|driver.py|timers.py|native.py', 40)
p.sort_stats('tottime').print_stats(25)
" > prof.txt 2>&1 && tail -n 1 perf.jsonl > summary.json && rm -rf ex64.bp prof.out
echo "exit $?"
