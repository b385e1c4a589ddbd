# Round 4 (final code): the driver's multi-rank commands on ONE GPU (ranks share the card: data
# path, tuning, phase profile and golden check -- not scaling): N=4, N=8, and BASELINE config 4
# (L=1024 fp64, 8 ranks).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4reh2}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/n4.json 2> $O/n4.err &&
timeout -k 10 500 python bench.py --gpus 8 --steps 20 --warmup 5 > $O/n8.json 2> $O/n8.err &&
timeout -k 10 600 python bench.py --gpus 8 --L 1024 --precision Float64 --steps 12 --warmup 3 > $O/n8_f64.json 2> $O/n8_f64.err
echo "exit $?"
