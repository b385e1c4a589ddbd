# Round 3: IPC unpack with 16 cells in flight per lane (GS_UNPACK_ITEMS=16, temporary override) vs 4, packed
# and z-plane ranks, overlapped and sequential passes, the exchange held >= GS_IPC_EMULATE_US; same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-unp3}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
for us in 0 30 60; do
  for mode in packed zplanes; do
    if [ $mode = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
    for ov in on off; do
      for it in 4 16; do
        GS_UNPACK_ITEMS=$it GS_IPC_EMULATE_US=$us timeout -k 10 120 python scripts/trace_overlap.py --mode $mode $A --passes 60 --overlap $ov --transport ipc > $O/tmp.txt 2>> $O/unp.err || { echo "run failed"; exit 1; }
        echo "emulate_us=$us items=$it $(cat $O/tmp.txt)" | tee -a $O/unp.txt
      done
    done
  done
done
