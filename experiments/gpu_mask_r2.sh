# Exec-masked Philox draw (ABL bit 32, exact): in-process A/B against the production tile, then a golden check.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-mask}
mkdir -p $O
cd $R
export GS_HIP_VARIANT=abl
timeout -k 10 300 python scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:1s 4x12:1s-abl32 --sched 2 --init random --rounds 6 --steps 60 > $O/ab_random.txt 2>&1 || { echo "ab random failed"; tail -n 20 $O/ab_random.txt; exit 1; }
timeout -k 10 300 python scripts/tune_inproc.py --L 512 --fuse 3 --cfg 4x12:1s 4x12:1s-abl32 --sched 2 --init seed --rounds 6 --steps 60 > $O/ab_seed.txt 2>&1 || { echo "ab seed failed"; exit 1; }
GS_FUSED_CFG=4x12:1s-abl32 GS_FUSED_SCHED=2 timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/bench_abl32.json 2> $O/bench_abl32.err || { echo "bench failed"; tail -n 5 $O/bench_abl32.err; exit 1; }
tail -n 12 $O/ab_random.txt
tail -n 12 $O/ab_seed.txt
python -c "import json; r=json.loads(open('$O/bench_abl32.json').read()); print(r['value'], r['config']['fused_kernel'], r['check'])"
