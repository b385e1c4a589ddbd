# Round 3: chained overlapped passes, shell_p beside inner_p (GS_OVERLAP_CHAIN=1) vs shell_p after
# inner_p (=2), against sequential passes, with the exchange held >= GS_IPC_EMULATE_US (IPC
# loopback, one MI355X); then kernel traces of both schedules at 30 us.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-chain3}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
for us in 0 30 60; do
  for mode in packed zplanes; do
    if [ $mode = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
    for ch in 1 2 off; do
      if [ $ch = off ]; then OV=off; C=1; else OV=on; C=$ch; fi
      GS_OVERLAP_CHAIN=$C GS_IPC_EMULATE_US=$us timeout -k 10 120 python scripts/trace_overlap.py --mode $mode $A --passes 60 --overlap $OV --transport ipc > $O/tmp.txt 2>> $O/emu.err || { echo "run failed $us $mode $ch"; exit 1; }
      echo "emulate_us=$us $(cat $O/tmp.txt)" | tee -a $O/emu.txt
    done
  done
done
for ch in 1 2; do
  GS_OVERLAP_CHAIN=$ch GS_IPC_EMULATE_US=30 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr$ch -o run -- python3 scripts/trace_overlap.py --mode packed --L 256 --nz 256 --passes 8 --overlap on --transport ipc > $O/tr$ch.log 2>&1 || { echo "trace failed $ch"; exit 1; }
  python3 scripts/trace_overlap.py --summarise $O/tr$ch > $O/trace_chain$ch.txt
done
echo done
