# Round 5, lease 9: output-step A/B in one box -- native vs torch snapshot call, queue depth.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c13}
mkdir -p $O
cd $R
export TMPDIR=/tmp
for v in "" "--queue 4"; do
  timeout -k 10 200 python scripts/profile_output.py --repeat 3 $v >> $O/output_ab.log 2>&1 || exit 1
done
timeout -k 10 60 python experiments/r5/write_probe.py /tmp >> $O/output_ab.log 2>&1
echo "exit $?"
