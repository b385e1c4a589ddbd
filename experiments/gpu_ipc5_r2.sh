# After the IPC poll refactor: IPC + loopback tests, smoke, the driver's bench command and the 2-rank torchrun.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-ipc5}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_rccl_loopback.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -n 30 $O/tests.log; exit 1; }
tail -n 1 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -n 1 $O/smoke.log &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 2 --steps 20 --warmup 5 > $O/torchrun2.json 2> $O/torchrun2.err
echo "exit $?"
python -c "import json; [print(f, r['value'], r['config']['transport'], r['check'].get('max_abs_err')) for f in ('bench', 'torchrun2') for r in [json.loads(open('$O/'+f+'.json').read())]]"
