# Round 5: the driver's multi-rank bench command rehearsed on ONE GPU (ranks share the card:
# data-path checks, not scaling numbers): N=2 and N=4 with the default tuning, N=2 with gated
# passes allowed on the shared card.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5rh}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err &&
timeout -k 10 500 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/n4.json 2> $O/n4.err &&
timeout -k 10 400 python bench.py --gpus 2 --steps 20 --warmup 5 --debug-knob gated=2 > $O/n2g.json 2> $O/n2g.err
echo "exit $?"
