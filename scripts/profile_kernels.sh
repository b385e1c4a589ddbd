#!/bin/bash
# Counter profile of the bench step (one counter group per rocprofv3 pass, kernel-trace only;
# never combined with sys/runtime traces).
# usage: scripts/profile_kernels.sh <outdir> [bench args...]
#   GS_FUSED_CFG / GS_FUSED_SCHED pin the fused kernel (otherwise the autotuner's candidates
#   show up as extra kernels with a few calls each).
set -e
out=${1:-gpurun_out/pmc}; shift || true
mkdir -p "$out"
export TMPDIR=/tmp
args="$@"
groups=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
  "FETCH_SIZE TCC_HIT_sum"
  "WRITE_SIZE TCC_MISS_sum"
  "SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
)
i=0
for g in "${groups[@]}"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $g --output-format csv -d "$out/g$i" -- python3 bench.py $args > "$out/g$i.log" 2>&1 || echo "group $i failed (counter unavailable?)"
  i=$((i+1))
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -- python3 bench.py $args > "$out/stats.log" 2>&1
echo "profile done"
