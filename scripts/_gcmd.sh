set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
cat gpurun_out/smoke.log | tail -2
timeout -k 10 300 python bench.py > gpurun_out/bench1.json 2> gpurun_out/bench1.err
cut -c1-300 gpurun_out/bench1.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof512 -o run -- python3 bench.py --steps 200 --warmup 20 > gpurun_out/prof512.log 2>&1
ls gpurun_out/prof512
