#!/bin/bash
# Sweep fused-kernel tile shapes and temporal depth on one GPU (L=512 fp32 bench config).
# usage: scripts/tune_fused.sh [outdir]
out=${1:-gpurun_out/tune}
mkdir -p "$out"
for fuse in 1 2 3; do
  for shape in 8x8 8x4 4x16 4x8; do
    if [ "$fuse" = 1 ] && [ "$shape" != 8x8 ]; then continue; fi
    GS_FUSED_SHAPE=$shape timeout -k 10 120 python bench.py --steps 120 --warmup 12 --fuse $fuse \
      > "$out/f${fuse}_${shape}.json" 2> "$out/f${fuse}_${shape}.err" || { echo "FAIL fuse=$fuse shape=$shape rc=$?"; exit 1; }
    python -c "import json,sys; d=json.load(open('$out/f${fuse}_${shape}.json')); print('fuse=$fuse shape=$shape', d['value'], 'MLUPS', d['ms_per_step'], 'ms/step', d['check'])"
  done
done
