set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/g5
mkdir -p $O
cd $R
for i in 1 2; do
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 --check none > $O/nochk_$i.json 2>/dev/null &&
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/chk_$i.json 2>/dev/null || exit 1
done
timeout -k 10 150 python bench.py --gpus 1 --steps 20 --warmup 50 --check none > $O/nochk_w50.json 2>/dev/null &&
timeout -k 10 150 python bench.py --gpus 1 --steps 200 --warmup 5 --check none > $O/nochk_s200.json 2>/dev/null &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof_nochk -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --check none > $O/prof_nochk.log 2>&1
echo "exit $?"
