set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6g}
mkdir -p $O
cd $R
GOLD=1 REPS=6 CFGS=4x8:1sl,4x8:1sl-w0,4x8:1sl-r3,4x8:1sl timeout -k 10 300 python -u experiments/r6/f64_lr_diag.py > $O/diag5.txt 2>&1 || { cat $O/diag5.txt; exit 1; }
cat $O/diag5.txt
