# IPC vs RCCL halo transport on one MI355X (loopback: a rank's periodic wraps to itself):
# wall time per overlapped / sequential pass, a kernel timeline of the IPC chain, and the
# driver's 2-rank torchrun bench on one GPU (RCCL refuses 2 ranks per device; IPC does not).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-ipcperf}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
for mode in zplanes packed; do
  if [ $mode = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
  for tr in rccl ipc; do
    for ov in on off; do
      timeout -k 10 120 python scripts/trace_overlap.py --mode $mode $A --passes 40 --overlap $ov --transport $tr >> $O/passes.txt 2>> $O/passes.err || { echo "pass run failed $mode $tr $ov"; exit 1; }
    done
  done
done
cat $O/passes.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tl_ipc -o run -- python3 $R/scripts/trace_overlap.py --mode zplanes --L 512 --nz 64 --passes 12 --transport ipc > $O/tl_ipc.log 2>&1 || { echo "trace failed"; exit 1; }
cd $R
python scripts/trace_overlap.py --summarise $O/tl_ipc > $O/tl_ipc_summary.txt 2>&1
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 20 --warmup 5 > $O/torchrun2.json 2> $O/torchrun2.err
echo "torchrun exit $?"
python -c "import json; r=json.loads(open('$O/torchrun2.json').read()); print(r['value'], r['config']['transport'], r['config']['dims'], r['tuning_s']); [print(x) for x in r['data_path_tuning']]"
