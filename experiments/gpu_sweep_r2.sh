# Full GPU test suite, then a bench.py sweep over grid sizes and precisions (one process each).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-sweep}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gputest.log 2>&1 || exit 1
run() { tag=$1; shift; timeout -k 10 200 python bench.py "$@" > $O/$tag.json 2> $O/$tag.err || exit 1; }
run L512_f32_driver --steps 20 --warmup 5
run L64_f32 --L 64 --steps 2000 --warmup 100
run L128_f32 --L 128 --steps 1000 --warmup 60
run L192_f32 --L 192 --steps 1000 --warmup 60
run L256_f32 --L 256 --steps 1000 --warmup 60
run L512_f32 --L 512 --steps 400 --warmup 40
run L1024_f32 --L 1024 --steps 60 --warmup 6
run L512_f64 --L 512 --precision Float64 --steps 200 --warmup 20
run L1024_f64 --L 1024 --precision Float64 --steps 30 --warmup 4
echo "exit 0"
