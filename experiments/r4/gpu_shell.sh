# Round 4: the x/y-only k_slab instantiation (<= 256 VGPRs) and the padded-row boundary fill:
# correctness tests, the one-sided 256^3 shell split, the driver's N=1 command.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4shell}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_overlap_shell.py tests/test_gpu_block.py tests/test_gpu_kernels.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 &&
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --one-sided --L 256 --nz 256 --k 3 2 --out $O/split_onesided.json > $O/split.log 2>&1 &&
timeout -k 10 300 python scripts/bench_overlap_split.py --packed --L 256 --nz 256 --k 3 --out $O/split_allsides.json >> $O/split.log 2>&1 &&
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err
echo "exit $?"
