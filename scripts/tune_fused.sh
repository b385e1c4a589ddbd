#!/bin/bash
# Sweep fused-kernel configurations (GS_FUSED_CFG=<rows>x<waves>:<prefetch>) and temporal
# depth on one GPU with the L=512 fp32 bench config.   usage: scripts/tune_fused.sh [outdir]
out=${1:-gpurun_out/tune}
mkdir -p "$out"
for fuse in ${FUSES:-2 3}; do
  for cfg in ${CFGS:-4x8:1 4x8:2 4x8:3 4x8:4 8x4:1 8x4:2 4x16:2 8x8:2}; do
    tag="f${fuse}_${cfg/:/_}"
    GS_FUSED_CFG=$cfg timeout -k 10 120 python bench.py --steps ${STEPS:-120} --warmup 12 --fuse $fuse \
      > "$out/$tag.json" 2> "$out/$tag.err" || { echo "FAIL fuse=$fuse cfg=$cfg rc=$?"; exit 1; }
    python -c "import json; d=json.load(open('$out/$tag.json')); print('fuse=$fuse cfg=$cfg', d['value'], 'MLUPS', d['ms_per_step'], 'ms/step')"
  done
done
