# Round 5, lease 3: neighbour-only LDS sync (FCfg::NSYNC) -- bitwise tests, in-process A/B in the
# driver's window at L=512 and at L=256, counters against the barrier tile, N=1 bench; the
# host-side output step of the reference example broken down (scripts/profile_output.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c3}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py -k "neighbour" -v --timeout 300 --timeout-method thread > $O/nsync_tests.log 2>&1 &&
timeout -k 10 600 python scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:1s 4x12:1sn 4x12:2s 4x12:2sn --sched 1 2 --init random --warmup 6 --steps 18 --rounds 5 --out $O/ab512.json > $O/ab512.log 2>&1 &&
timeout -k 10 600 python scripts/tune_inproc.py --L 256 --fuse 3 --cfg 4x12:1sf 4x12:1sfn --sched 1 2 --init random --warmup 6 --steps 30 --rounds 5 --out $O/ab256.json > $O/ab256.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "fp64_lds" -v --timeout 300 --timeout-method thread > $O/f64_tests.log 2>&1 &&
timeout -k 10 600 python scripts/tune_inproc.py --precision Float64 --L 512 1024 --fuse 3 --cfg 4x8:1s 4x8:1sn 4x8:1sxn --sched 2 --init random --warmup 6 --steps 30 --rounds 3 --out $O/ab_f64.json > $O/ab_f64.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/n1b.json 2> $O/n1b.err &&
PIN_TILE=4x12:1s PIN_SCHED=1 bash scripts/pmc_pinned.sh $O/pmc_bar $O/n1.json --steps 21 --warmup 6 &&
PIN_TILE=4x12:1sn PIN_SCHED=1 bash scripts/pmc_pinned.sh $O/pmc_nsync $O/n1.json --steps 21 --warmup 6 &&
timeout -k 10 300 python scripts/profile_output.py --repeat 3 > $O/output_prof.log 2>&1
echo "exit $?"
