# Round 4: rehearsal of the driver's multi-rank commands on ONE GPU (the ranks share the card, so
# these check the data path, tuning, per-phase profile and golden check -- not scaling), N=4 and 8.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4reh}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/n4.json 2> $O/n4.err &&
timeout -k 10 500 python bench.py --gpus 8 --steps 20 --warmup 5 > $O/n8.json 2> $O/n8.err
echo "exit $?"
