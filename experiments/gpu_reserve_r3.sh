# Round 3: workgroup slots the overlapped inner launch leaves free for the comm chain (signal/wait,
# unpack, face-slab shell), after the cell-granular split: 16 (the constant) vs 48 / 96, with the
# IPC loopback exchange held >= GS_IPC_EMULATE_US; sequential passes for reference.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-res3}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
for us in 0 30 60; do
  for mode in packed zplanes; do
    if [ $mode = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
    GS_IPC_EMULATE_US=$us timeout -k 10 120 python scripts/trace_overlap.py --mode $mode $A --passes 60 --overlap off --transport ipc > $O/tmp.txt 2>> $O/res.err || { echo "run failed"; exit 1; }
    echo "emulate_us=$us reserve=- $(cat $O/tmp.txt)" | tee -a $O/res.txt
    for r in 16 48 96; do
      GS_OVERLAP_RESERVE=$r GS_IPC_EMULATE_US=$us timeout -k 10 120 python scripts/trace_overlap.py --mode $mode $A --passes 60 --overlap on --transport ipc > $O/tmp.txt 2>> $O/res.err || { echo "run failed"; exit 1; }
      echo "emulate_us=$us reserve=$r $(cat $O/tmp.txt)" | tee -a $O/res.txt
    done
  done
done
