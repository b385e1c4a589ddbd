# Round 6: link probe + model pruning and the config-3 geometry bitwise test
# (item 5) on one GPU; then the driver's multi-rank command rehearsed on one card
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6q}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_linkprobe.py tests/test_gpu_gated.py -k "link_probe or config3" -x -v -s --timeout 400 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -3 $O/pytest.txt
for n in 2 4; do
  timeout -k 10 400 python bench.py --gpus $n --steps 20 --warmup 5 > $O/b$n.json 2> $O/b$n.err || { tail -20 $O/b$n.err; exit 1; }
  python scripts/rehearsal_row.py $O/b$n.json | tee -a $O/summary.txt
done
timeout -k 10 500 python bench.py --gpus 8 --steps 20 --warmup 5 --debug-knob gated=2 > $O/b8g.json 2> $O/b8g.err || { tail -20 $O/b8g.err; exit 1; }
python scripts/rehearsal_row.py $O/b8g.json | tee -a $O/summary.txt
