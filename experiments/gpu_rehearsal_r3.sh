# The driver's SCALE commands rehearsed on ONE GPU with the default transport (auto: the IPC
# candidates are in the list): N ranks share the card, so RCCL refuses and the tuning falls back
# per candidate; the point is the tuning wall time, the table and every failed row's reason.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-reh3}
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 420 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err &&
timeout -k 10 420 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/n4.json 2> $O/n4.err &&
timeout -k 10 480 python bench.py --gpus 8 --steps 20 --warmup 5 > $O/n8.json 2> $O/n8.err
echo "exit $?"
