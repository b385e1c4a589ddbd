set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${GS_OUT:-r6t64}
mkdir -p $O
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -- python3 bench.py --gpus 1 --L 64 --steps 300 --warmup 30 --profile-passes 0 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 - $O/trace <<'PY' | tee $O/gaps.txt
import csv, glob, os, sys
rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
rows.sort()
st = [i for i, r in enumerate(rows) if "k_stats" in r[2]]
end = st[0] if st else len(rows)
win = rows[max(0, end - 100):end]
gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(win, win[1:])]
durs = [(e - s) / 1e3 for s, e, _ in win]
import statistics as S
print(f"last 100 dispatches before k_stats: kernel us median {S.median(durs):.2f}, gap us median {S.median(gaps):.2f} mean {S.mean(gaps):.2f} max {max(gaps):.2f}")
print("kernels:", sorted(set(n for _, _, n in win)))
PY
