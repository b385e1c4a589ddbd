#!/bin/bash
# Strong-scaling sweep of the headline benchmark (L=512 fp32) on 1/2/4/8 GPUs of one node.
#   scripts/bench_scaling.sh [steps] [warmup]
set -e
here=$(cd "$(dirname "$0")" && pwd)
source "$here/env_mi355x.sh"
steps=${1:-400}; warmup=${2:-40}
for n in 1 2 4 8; do
  if [ "$n" = 1 ]; then
    python "$here/../bench.py" --steps "$steps" --warmup "$warmup"
  else
    python -m torch.distributed.run --nnodes 1 --nproc-per-node $n --master-addr 127.0.0.1 \
      --master-port $((29600 + n)) "$here/../bench.py" --gpus $n --steps "$steps" --warmup "$warmup"
  fi
done
