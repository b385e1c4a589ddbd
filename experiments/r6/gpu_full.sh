# Round 6 re-entry: full GPU test suite, smoke, the driver's bench command x3, K=400
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6final}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=5 -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b20_$i.json 2> $O/b20_$i.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); c=d['config']; print('K=20', d['value'], d['ms_per_step'], c.get('pass_plan'), c.get('fused_kernel'), d['check'].get('golden_ok'))" $O/b20_$i.json | tee -a $O/summary.txt
done
