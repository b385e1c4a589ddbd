#!/bin/bash
# Run one simulation on the GPUs of ONE node: one rank per MI355X.
#   scripts/run_node.sh <settings.toml> [ngpus]
# (reference launchers: srun -n 1 --gpus=1 / jsrun / mpirun, scripts/job_*.sh)
set -e
here=$(cd "$(dirname "$0")" && pwd)
source "$here/env_mi355x.sh"
cfg=${1:?settings file}
n=${2:-$(python -c 'import torch; print(torch.cuda.device_count())')}
exec python -m torch.distributed.run --nnodes 1 --nproc-per-node "$n" \
  --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29513} "$here/../gray-scott.py" "$cfg"
