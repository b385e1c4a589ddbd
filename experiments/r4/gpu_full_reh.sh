# Round 4: the full check (experiments/r4/gpu_full.sh), the N=4 / N=8 one-GPU rehearsal, an A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash experiments/r4/gpu_full.sh | grep -q "exit 0" && GS_OUT=r4reh bash experiments/r4/gpu_rehearsal.sh | grep -q "exit 0" && bash experiments/r4/gpu_ab2.sh
echo "exit $?"
