# Round 3: the packed 256^3 overlap at fuse depth 2 (shell 11 us instead of 28) vs depth 3, with the
# exchange emulated on the IPC loopback (per pass and per step).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-emu3k2}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
for us in 0 30 60; do
  for k in 2 3; do
    for ov in on off; do
      GS_IPC_EMULATE_US=$us timeout -k 10 120 python scripts/trace_overlap.py --mode packed --L 256 --nz 256 --fuse $k --passes 60 --overlap $ov --transport ipc > $O/tmp.txt 2>> $O/emu.err || { echo "run failed $us $k $ov"; exit 1; }
      echo "emulate_us=$us $(cat $O/tmp.txt)" | tee -a $O/emu.txt
    done
  done
done
