# Round 4 final check: GPU suite, smoke, the driver's N=1 command twice, bench default (400 steps),
# L=256 (BASELINE config 2), the 2-rank command (ranks share the card).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4final}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv1.json 2> $O/drv1.err &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv2.json 2> $O/drv2.err &&
timeout -k 10 300 python bench.py > $O/l512.json 2> $O/l512.err &&
timeout -k 10 200 python bench.py --L 256 --steps 1000 --warmup 100 > $O/l256.json 2> $O/l256.err &&
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err
echo "exit $?"
