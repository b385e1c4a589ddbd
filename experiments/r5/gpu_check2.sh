# Round 5, lease 2: the reference-length parity runs (drift numbers printed), the fp64 LDS
# x-sum tiles (bitwise tests, in-process A/B, bench at L=512 / 1024, counters), the GPU suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c2}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_oracle.py tests/test_gpu_kernels.py -k "julia or fp64_lds or oracle" -v -s --timeout 300 --timeout-method thread > $O/oracle.log 2>&1 &&
timeout -k 10 600 python scripts/tune_inproc.py --precision Float64 --L 512 1024 --fuse 3 --cfg 4x8:1s 4x8:1sx 4x6:2sx 4x8:1x --sched 1 2 --init random --warmup 6 --steps 30 --rounds 3 --out $O/ab_f64.json > $O/ab_f64.log 2>&1 &&
timeout -k 10 300 python bench.py --precision Float64 --L 512 --steps 30 --warmup 6 > $O/f64_512.json 2> $O/f64_512.err &&
timeout -k 10 300 python bench.py --precision Float64 --L 1024 --steps 12 --warmup 3 > $O/f64_1024.json 2> $O/f64_1024.err &&
bash scripts/pmc_pinned.sh $O/pmc_f64_1024 $O/f64_1024.json --precision Float64 --L 1024 --steps 6 --warmup 3 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputests.log 2>&1
echo "exit $?"
