# Round 4: counters of the production T=3 kernel with the step-uniform Philox words in VGPRs (PU)
# against the PU-off ablation (4x12:1s-abl256), L=512 fp32, the driver's window; HBM bytes in
# their own passes; then the host write probe of the BP4 output step.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-roof4}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export GS_FUSED_SCHED=2
SQ="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY"
GS_FUSED_CFG=4x12:1s timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/trace.log 2>&1 &&
GS_FUSED_CFG=4x12:1s timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/fetch.log 2>&1 &&
GS_FUSED_CFG=4x12:1s timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/write.log 2>&1 &&
GS_FUSED_CFG=4x12:1s timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d $O/sq -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/sq.log 2>&1 &&
GS_HIP_VARIANT=abl GS_FUSED_CFG=4x12:1s-abl256 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $SQ --output-format csv -d $O/sq_pu_off -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/sq_pu_off.log 2>&1 &&
GS_HIP_VARIANT=abl GS_FUSED_CFG=4x12:1s-abl256 timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_pu_off -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/trace_pu_off.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/grbm -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/grbm.log 2>&1 &&
cd $O && g++ -O2 -pthread -o /tmp/write_probe $R/csrc/tools/write_probe.cpp && timeout -k 10 120 /tmp/write_probe 1 > $O/write_probe.txt 2>&1
echo "exit $?"
