# Multi-rank rehearsal on ONE GPU: N ranks share the card (RCCL refuses duplicate GPUs, so the
# host transport carries the halos); checks the self-launch, data-path tuning budget and report.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-reh}
mkdir -p $O
cd $R
timeout -k 10 420 python bench.py --gpus 8 --steps 20 --warmup 5 --transport host > $O/r8_host.json 2> $O/r8_host.err &&
GS_COMM_TIMEOUT=60 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/r2_auto.json 2> $O/r2_auto.err
echo "exit $?"
