# Round 4: inter-kernel gap of back-to-back fused passes by grid size (kernel traces of bench.py,
# pinned 4x12:1s schedule 2): is it the kernel-end L2 writeback (scales with dirty bytes)?
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4gap}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for L in 128 192 256 384; do
  GS_FUSED_CFG=4x12:1s GS_FUSED_SCHED=2 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$L -o run -- python3 $R/bench.py --L $L --fuse 3 --steps 60 --warmup 6 --check none > $O/tr_$L.log 2>&1 || exit 1
done
echo "exit $?"
