# Round 5, first lease: the GPU suite with the non-blocking RCCL set-up (loopback, IPC,
# multi-rank, first contact), the driver's N=1 command, fp64 L=512 / L=1024, and counters of
# the chosen fp64 and fp32 kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r5c1}
mkdir -p $O
cd $R
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gputests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/n1.json 2> $O/n1.err &&
timeout -k 10 300 python bench.py --precision Float64 --L 512 --steps 30 --warmup 6 > $O/f64_512.json 2> $O/f64_512.err &&
timeout -k 10 300 python bench.py --precision Float64 --L 1024 --steps 12 --warmup 3 > $O/f64_1024.json 2> $O/f64_1024.err &&
bash scripts/pmc_pinned.sh $O/pmc_f64_512 $O/f64_512.json --precision Float64 --L 512 --steps 15 --warmup 3 &&
bash scripts/pmc_pinned.sh $O/pmc_f64_1024 $O/f64_1024.json --precision Float64 --L 1024 --steps 6 --warmup 3 &&
bash scripts/pmc_pinned.sh $O/pmc_f32_512 $O/n1.json --steps 21 --warmup 6
echo "exit $?"
