# Cross-stream event scope (GS_XSTREAM_EVENT 0 system / 1 device release / 2 no system fence): chained
# overlapped passes through the RCCL and IPC loopback, interleaved, then the loopback tests under the faster mode.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-xevent}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
for rep in 1 2; do
for xm in 0 1 2; do
  for tr in rccl ipc; do
    for mode in zplanes packed; do
      if [ $mode = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
      GS_XSTREAM_EVENT=$xm timeout -k 10 120 python scripts/trace_overlap.py --mode $mode $A --passes 40 --overlap on --transport $tr > $O/tmp.txt 2>> $O/err.txt || { echo "run failed"; exit 1; }
      echo "xevent=$xm $(cat $O/tmp.txt)" | tee -a $O/passes.txt
    done
  done
done
done
for xm in 1 2; do
  GS_XSTREAM_EVENT=$xm timeout -k 10 400 python -u -m pytest tests/test_gpu_ipc.py tests/test_gpu_rccl_loopback.py -x -q --timeout 120 --timeout-method thread > $O/tests_$xm.log 2>&1 || { echo "tests failed xevent=$xm"; tail -n 20 $O/tests_$xm.log; exit 1; }
  tail -n 1 $O/tests_$xm.log
done
