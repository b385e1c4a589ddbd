# Round 5: the driver's short bench (K=20, W=5) vs longer warm-ups / timed regions, 3 runs each
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5kw}
mkdir -p $O
cd $R
for kw in "20 5" "20 50" "21 5" "18 5" "200 5" "20 5"; do
  set -- $kw
  for i in 1 2; do
    timeout -k 10 200 python bench.py --gpus 1 --steps $1 --warmup $2 > $O/b_${1}_${2}_$i.json 2> $O/b_${1}_${2}_$i.err || exit 1
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" $O/b_${1}_${2}_$i.json $1 $2 | tee -a $O/summary.txt
  done
done
