set -e
mkdir -p gpurun_out
for dv in 0 4 2 1; do
for L in 64 128 256; do
GS_FUSED_CHDIV=$dv timeout -k 10 120 python bench.py --L $L --steps 600 --warmup 60 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('chdiv $dv L',d['config']['L'],'fuse',d['config']['fuse_steps'],'us/step',round(d['ms_per_step']*1000,2),'MLUPS',d['value'], d['config']['fused_kernel'])"
done
GS_FUSED_CHDIV=$dv timeout -k 10 120 python scripts/bench_overlap_split.py --L 512 --nz 64 --k 2 3 2>/dev/null | grep "^{" | cut -c1-120
done
