# Counters of the pinned production fused kernels (one rocprofv3 pass each, kernel-trace only),
# the RCCL-loopback overlap timelines, and a 2-rank transport-fallback rehearsal.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-pmc}
mkdir -p $O
cd $R
GS_COMM_TIMEOUT=60 timeout -k 10 300 python bench.py --gpus 2 --steps 20 --warmup 5 > $O/r2_auto.json 2> $O/r2_auto.err || echo "2-rank auto rehearsal failed: $?"
cd /tmp && export TMPDIR=/tmp
for cfg in 4x12:2s 4x12:1s; do
  tag=${cfg//:/_}
  GS_FUSED_CFG=$cfg GS_FUSED_SCHED=2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc_$tag -o run -- python3 $R/bench.py --steps 20 --warmup 5 --check none > $O/pmc_$tag.log 2>&1 || { echo "pmc $cfg failed"; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/ovl_z -o run -- python3 $R/scripts/trace_overlap.py --mode zplanes --L 512 --nz 64 > $O/ovl_z.log 2>&1 &&
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/ovl_p -o run -- python3 $R/scripts/trace_overlap.py --mode packed --L 256 --nz 256 > $O/ovl_p.log 2>&1
echo "exit $?"
