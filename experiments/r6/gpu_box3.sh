#!/bin/bash
# The driver's command three times on one fresh box (final tree).
set -o pipefail
O=gpurun_out/${GS_OUT:-r6box}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b$i.json 2> $O/b$i.err || { tail -20 $O/b$i.err; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['config']['pass_plan'], d['check']['golden_ok'], [w.get('pci') for w in d['world']['per_rank']])" $O/b$i.json
done
