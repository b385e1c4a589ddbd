# Round 3: the T=3 production fused kernel's HBM roofline at L=512 fp32:
# FETCH_SIZE and WRITE_SIZE in their own passes (TCC budget), kernel durations from a trace,
# VALU counts; the production tile pinned (4x12:1s, schedule 2).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-roof3}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GS_FUSED_CFG=4x12:1s GS_FUSED_SCHED=2
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/write.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY --output-format csv -d $O/sq -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/sq.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/grbm -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/grbm.log 2>&1
echo "exit $?"
