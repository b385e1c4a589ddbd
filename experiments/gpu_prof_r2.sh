# Final-kernel profile: rocprofv3 kernel stats of the driver's bench command, and one SQ counter pass of the
# pinned production kernels (4x12:1s T=3 / T=2, schedule 2), each in its own run.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-prof}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o run -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 > $O/stats.log 2>&1 || { echo "stats failed"; exit 1; }
GS_FUSED_CFG=4x12:1s GS_FUSED_SCHED=2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD --output-format csv -d $O/pmc -o run -- python3 $R/bench.py --steps 20 --warmup 5 --check none > $O/pmc.log 2>&1 || { echo "pmc failed"; exit 1; }
GS_FUSED_CFG=4x12:1s GS_FUSED_SCHED=2 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc2 -o run -- python3 $R/bench.py --steps 20 --warmup 5 --check none > $O/pmc2.log 2>&1
echo "exit $?"
