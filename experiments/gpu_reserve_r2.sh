# Workgroup slots the overlapped inner launch leaves free (GS_OVERLAP_RESERVE) with the IPC and RCCL loopback.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-reserve}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
for rep in 1 2; do
for rs in 0 8 16 32; do
  for tr in ipc rccl; do
    for mode in zplanes packed; do
      if [ $mode = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
      GS_OVERLAP_RESERVE=$rs timeout -k 10 120 python scripts/trace_overlap.py --mode $mode $A --passes 40 --overlap on --transport $tr > $O/tmp.txt 2>> $O/err.txt || { echo "run failed"; exit 1; }
      echo "reserve=$rs $(grep us_per_pass $O/tmp.txt)" | tee -a $O/passes.txt
    done
  done
done
done
