set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/g2
cd $R
timeout -k 10 120 python scripts/power_probe.py --passes 60 > gpurun_out/g2/probe.txt 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU --output-format csv -d $R/gpurun_out/g2/pmc -o run -- python3 $R/scripts/power_probe.py --passes 30 > $R/gpurun_out/g2/pmc.log 2>&1
echo "exit $?"
