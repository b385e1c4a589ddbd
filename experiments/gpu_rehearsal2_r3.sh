# Round 3: the driver's SCALE commands on ONE GPU (N ranks share the card) with the current code,
# plus the 8-rank fp64 L=512 run whose post-timing golden check covers the fp64 multi-rank path.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-reh3b}
mkdir -p $O
cd $R
timeout -k 10 420 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/n2.json 2> $O/n2.err &&
timeout -k 10 420 python bench.py --gpus 4 --steps 20 --warmup 5 > $O/n4.json 2> $O/n4.err &&
timeout -k 10 480 python bench.py --gpus 8 --steps 20 --warmup 5 > $O/n8.json 2> $O/n8.err &&
timeout -k 10 480 python bench.py --gpus 8 --steps 20 --warmup 5 --precision Float64 --L 512 > $O/n8_f64.json 2> $O/n8_f64.err
echo "exit $?"
