# Round 4: where the production kernel's wave-cycles go (SQ counters, one pass per group of 8),
# L=512 fp32 T=3, 4x12:1s schedule 2, the driver's window.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4stall}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GS_FUSED_CFG=4x12:1s GS_FUSED_SCHED=2
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT --output-format csv -d $O/p1 -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $O/p2 -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/p2.log 2>&1
echo "exit $?"
