# Round 3: overlapped vs sequential passes with a slow exchange, after the cell-granular split:
# the IPC loopback with every exchange held for at least GS_IPC_EMULATE_US (a stand-in for an
# xGMI transfer), one MI355X.  packed = 256^3 with neighbours on all 26 sides; zplanes = 512^2x64.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-emu3}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
for us in 0 30 60 100; do
  for mode in packed zplanes; do
    if [ $mode = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
    for ov in on off; do
      GS_IPC_EMULATE_US=$us timeout -k 10 120 python scripts/trace_overlap.py --mode $mode $A --passes 60 --overlap $ov --transport ipc > $O/tmp.txt 2>> $O/emu.err || { echo "run failed $us $mode $ov"; exit 1; }
      echo "emulate_us=$us $(cat $O/tmp.txt)" | tee -a $O/emu.txt
    done
  done
done
