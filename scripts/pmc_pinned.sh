#!/bin/bash
# Counter passes of the fused kernel a bench.py run chose, pinned so no autotuner candidate
# shows up: one rocprofv3 pass per counter group (kernel-trace only, never with sys/runtime
# traces), then the kernel statistics, then the per-dispatch summary (scripts/pmc_summary.py).
# usage: scripts/pmc_pinned.sh <outdir> <bench json> [bench args...]
#   the bench json names the tile / schedule per depth (config.fused_kernel); the deepest depth
#   is pinned through GS_FUSED_CFG / GS_FUSED_SCHED.
set -o pipefail
out=$1; js=$2; shift 2
mkdir -p "$out"
export TMPDIR=/tmp
read -r tile sched < <(python3 - "$js" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
fk = d["config"]["fused_kernel"]
c = fk[max(fk, key=int)]
print(c["tile"] if c["tile"] != "default" else "-", c["sched"])
PY
) || exit 1
# PIN_TILE / PIN_SCHED override the bench's choice (A/B counter sets of two tiles)
tile=${PIN_TILE:-$tile}; sched=${PIN_SCHED:-$sched}
if [ "$tile" != "-" ]; then export GS_FUSED_CFG=$tile; fi
export GS_FUSED_SCHED=$sched GS_AUTOTUNE=0
echo "pinned tile=$tile sched=$sched" | tee "$out/pinned.txt"
groups=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
  "FETCH_SIZE TCC_HIT_sum"
  "WRITE_SIZE TCC_MISS_sum"
)
i=0
for g in "${groups[@]}"; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $g --output-format csv -d "$out/g$i" -- python3 bench.py --check none --profile-passes 0 "$@" > "$out/g$i.log" 2>&1 || { echo "group $i failed"; exit 1; }
  i=$((i+1))
done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -- python3 bench.py --check none --profile-passes 0 "$@" > "$out/stats.log" 2>&1 || exit 1
python3 scripts/pmc_summary.py "$out" > "$out/summary.txt"
echo "pmc done: $out"
