# Round 4: A/B of the Philox blocks drawn before the workgroup barrier (-abl512 all levels,
# -abl1024 top level, -abl1536 top two) against the production 4x12:1s, L=512 / L=256 T=3.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r4hoist}
mkdir -p $O
cd $R
GS_HIP_VARIANT=abl timeout -k 10 600 python scripts/tune_inproc.py --L 512 --fuse 3 --init random --warmup 6 --steps 18 --rounds 5 --sched 1 2 --cfg 4x12:1s 4x12:1s-abl512 4x12:1s-abl1024 4x12:1s-abl1536 --out $O/ab512.json > $O/ab512.log 2>&1 &&
GS_HIP_VARIANT=abl timeout -k 10 600 python scripts/tune_inproc.py --L 256 --fuse 3 --init random --warmup 10 --steps 60 --rounds 5 --sched 1 2 --cfg 4x12:1s 4x12:1s-abl512 4x12:1s-abl1024 4x12:1s-abl1536 --out $O/ab256.json > $O/ab256.log 2>&1
echo "exit $?"
# the reference's L=64 example under cProfile: where the 0.44 ms per output step goes
mkdir -p $O/ex64 && cd $O/ex64 && sed -e 's/^output = .*/output = "ex64.bp"/' $R/examples/settings-files.toml > ex.toml &&
echo 'perf_log = "perf-ex64.jsonl"' >> ex.toml &&
timeout -k 10 300 python3 -m cProfile -o prof.out $R/gray-scott.py ex.toml > ex.log 2> ex.err &&
python3 -c "import pstats; p=pstats.Stats('prof.out'); p.sort_stats('tottime').print_stats(30); p.sort_stats('cumulative').print_stats(40)" > prof.txt 2>&1 &&
tail -n 1 perf-ex64.jsonl > summary.json && rm -rf ex64.bp prof.out
echo "exit $?"
