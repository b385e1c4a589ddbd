set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/pmc_final
GS_FUSED_CFG=4x12:1s GS_FUSED_SCHED=2 timeout -k 10 900 bash scripts/profile_kernels.sh gpurun_out/pmc_final --steps 60 --warmup 6 > gpurun_out/pmc_final.log 2>&1
python scripts/pmc_summary.py gpurun_out/pmc_final > gpurun_out/pmc_final_summary.txt
grep -A22 "k_fused" gpurun_out/pmc_final_summary.txt | head -24
