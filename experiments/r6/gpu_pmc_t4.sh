# Round 6: counter table of the T=4 LDS-ring dispatch (4x12:1sfl, sched 2) at L=512 fp32, pinned
# (FETCH/WRITE, VALU, SQ_WAIT_ANY, TCC_HIT/MISS, SQ_LDS_BANK_CONFLICT), and the
# T=3 register-ring dispatch (4x12:1s) on the same box for the A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6p}
mkdir -p $O
cd $R
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --fuse 4 > $O/b_t4.json 2> $O/b_t4.err || exit 1
PIN_TILE=4x12:1sfl PIN_SCHED=2 timeout -k 10 900 bash scripts/pmc_pinned.sh $O/t4 $O/b_t4.json --gpus 1 --fuse 4 --steps 40 --warmup 8 || exit 1
PIN_TILE=4x12:1s PIN_SCHED=2 timeout -k 10 900 bash scripts/pmc_pinned.sh $O/t3 $O/b_t4.json --gpus 1 --fuse 3 --steps 42 --warmup 9 || exit 1
cat $O/t4/summary.txt $O/t3/summary.txt
