# IPC transport after dropping the redundant slot-release flags: tests, then the per-pass A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-ipc2}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipc.py -x -v --timeout 120 --timeout-method thread > $O/ipc.log 2>&1 || { echo "ipc tests failed"; tail -n 30 $O/ipc.log; exit 1; }
tail -n 2 $O/ipc.log
GS_OUT=${GS_OUT:-ipc2} bash experiments/gpu_ipc_perf_r2.sh
cd $R
timeout -k 10 400 python bench.py --gpus 4 --steps 20 --warmup 5 --timeout 380 > $O/selflaunch4.json 2> $O/selflaunch4.err
echo "selflaunch4 exit $?"
python -c "import json; r=json.loads(open('$O/selflaunch4.json').read()); print(r['value'], r['config']['transport'], r['config']['dims'], r['tuning_s'], r['wall_s']); [print(x) for x in r['data_path_tuning']]"
