# Round 3: the IPC receive side as one signal + wait + unpack launch (k_ipc_wait_unpack) with
# G workgroups vs separate signal-wait and unpack launches (G=0), overlapped chain, emulated
# exchange (IPC loopback, one MI355X); IPC tests first.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-unpack3}
mkdir -p $O
cd $R
export GS_COMM_TIMEOUT=60
timeout -k 10 400 python -u -m pytest tests/test_gpu_ipc.py -x -v --timeout 300 --timeout-method thread > $O/ipc_tests.log 2>&1 || { echo "ipc tests failed"; exit 1; }
for us in 0 30 60; do
  for mode in packed zplanes; do
    if [ $mode = zplanes ]; then A="--L 512 --nz 64"; else A="--L 256 --nz 256"; fi
    for G in 0 32 64 128 256 off; do
      if [ $G = off ]; then OV=off; GG=64; else OV=on; GG=$G; fi
      GS_IPC_UNPACK_GROUPS=$GG GS_IPC_EMULATE_US=$us timeout -k 10 120 python scripts/trace_overlap.py --mode $mode $A --passes 60 --overlap $OV --transport ipc > $O/tmp.txt 2>> $O/emu.err || { echo "run failed $us $mode $G"; exit 1; }
      echo "emulate_us=$us groups=$G $(cat $O/tmp.txt)" | tee -a $O/emu.txt
    done
  done
done
for G in 64 128; do
  GS_IPC_UNPACK_GROUPS=$G GS_IPC_EMULATE_US=30 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr$G -o run -- python3 scripts/trace_overlap.py --mode packed --L 256 --nz 256 --passes 8 --overlap on --transport ipc > $O/tr$G.log 2>&1 || { echo "trace failed $G"; exit 1; }
  python3 scripts/trace_overlap.py --summarise $O/tr$G > $O/trace_g$G.txt
done
echo done
