# Round 6: kernel timeline of the driver's command (K=20, W=5) under rocprofv3 --kernel-trace --stats
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6t}
mkdir -p $O
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 scripts/trace_window.py $O/trace > $O/timeline.txt || exit 1
cat $O/timeline.txt
