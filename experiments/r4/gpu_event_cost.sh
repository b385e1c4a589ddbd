# Round 4: stream-time cost of event records between fused passes (scripts/event_cost.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4evcost}
mkdir -p $O
cd $R
timeout -k 10 300 python scripts/event_cost.py --L 256 --passes 40 --rounds 5 > $O/ev256.log 2>&1 &&
timeout -k 10 300 python scripts/event_cost.py --L 128 --passes 60 --rounds 5 > $O/ev128.log 2>&1
echo "exit $?"
