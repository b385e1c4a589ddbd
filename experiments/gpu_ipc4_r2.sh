# NOTE: the wide-copy path (GS_IPC_COPY_RUNS) was rejected and removed (profiles/r2_ipc_copy_rejected.txt); kept as the record of how it was measured.
# IPC z-plane plans through the wide contiguous copy (k_copy_runs) vs the cell-wise pack kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-ipc4}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
timeout -k 10 300 python -u -m pytest tests/test_gpu_ipc.py -x -v --timeout 120 --timeout-method thread > $O/ipc.log 2>&1 || { echo "ipc tests failed"; tail -n 30 $O/ipc.log; exit 1; }
tail -n 1 $O/ipc.log
for cr in 1 0 1 0; do
  for ov in on off; do
    GS_IPC_COPY_RUNS=$cr timeout -k 10 120 python scripts/trace_overlap.py --mode zplanes --L 512 --nz 64 --passes 40 --overlap $ov --transport ipc > $O/tmp.txt 2>> $O/err.txt || { echo "run failed"; exit 1; }
    echo "copy_runs=$cr $(cat $O/tmp.txt)" | tee -a $O/passes.txt
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tl -o run -- python3 $R/scripts/trace_overlap.py --mode zplanes --L 512 --nz 64 --passes 12 --transport ipc --overlap off > $O/tl.log 2>&1 || { echo "trace failed"; exit 1; }
cd $R
python scripts/trace_overlap.py --summarise $O/tl > $O/tl_summary.txt 2>&1
tail -n 8 $O/tl_summary.txt
