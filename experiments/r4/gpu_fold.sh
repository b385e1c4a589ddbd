# Round 4: the folded last x strip (4x12:1sf): correctness (golden + bitwise vs 4x12:1s), in-process
# A/B at L=256 / 192 / 128, and bench.py at L=256 / 128 (autotuned: the tuner may pick it).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4fold}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py -m gpu -x -q -k "folded" --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python scripts/tune_inproc.py --L 256 --fuse 3 --init random --warmup 10 --steps 60 --rounds 5 --sched 1 2 --cfg 4x12:1s 4x12:1sf --out $O/ab256.json > $O/ab256.log 2>&1 &&
timeout -k 10 300 python scripts/tune_inproc.py --L 192 --fuse 3 --init random --warmup 10 --steps 90 --rounds 5 --sched 1 2 --cfg 4x12:1s 4x12:1sf --out $O/ab192.json > $O/ab192.log 2>&1 &&
timeout -k 10 300 python scripts/tune_inproc.py --L 128 --fuse 3 --init random --warmup 10 --steps 150 --rounds 5 --sched 1 2 --cfg 4x12:1s 4x12:1sf --out $O/ab128.json > $O/ab128.log 2>&1 &&
timeout -k 10 200 python bench.py --L 256 --steps 1000 --warmup 100 > $O/l256.json 2> $O/l256.err &&
timeout -k 10 200 python bench.py --L 128 --steps 1000 --warmup 100 > $O/l128.json 2> $O/l128.err
echo "exit $?"
