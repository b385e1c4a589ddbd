set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6x}
mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_$i.json 2> $O/b20_$i.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('K=20', d['value'], d['ms_per_step'], c.get('pass_plan'), d['check'].get('golden_ok'), d['world']['per_rank'][0].get('pci'))" $O/b20_$i.json | tee -a $O/summary.txt
done
