# Round 4: output-store cache policy (-abl2048 nt, -abl4096 sc1 = device scope / write-through,
# -abl6144 both) against the production 4x12:1s: in-process A/B at L=512 T=3, then kernel traces
# of the driver's window to read the inter-kernel gap (kernel-end L2 writeback).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4store}
mkdir -p $O
cd $R
GS_HIP_VARIANT=abl timeout -k 10 600 python scripts/tune_inproc.py --L 512 --fuse 3 --init random --warmup 6 --steps 18 --rounds 5 --sched 2 --cfg 4x12:1s 4x12:1s-abl2048 4x12:1s-abl4096 4x12:1s-abl6144 --out $O/ab512.json > $O/ab512.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
for c in 4x12:1s 4x12:1s-abl2048 4x12:1s-abl4096 4x12:1s-abl6144; do
  t=${c//:/_}
  GS_HIP_VARIANT=abl GS_FUSED_CFG=$c GS_FUSED_SCHED=2 timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$t -o run -- python3 $R/bench.py --steps 21 --warmup 6 --check none > $O/tr_$t.log 2>&1 || exit 1
done
echo "exit $?"
