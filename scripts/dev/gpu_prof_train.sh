#!/bin/bash
# rocprof kernel breakdown of the C2 1vsAll training step (replayed HIP graph).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_train -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/prof_train.py complex 1vsAll > $GRAFT_REPO_ROOT/gpurun_out/prof_train.log 2>&1 || { echo "failed"; tail $GRAFT_REPO_ROOT/gpurun_out/prof_train.log; exit 1; }
cd $GRAFT_REPO_ROOT
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/prof_train/**/run_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':70s} calls   avg_us   pct")
for r in rows[:24]:
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:8.1f} {100*float(r['TotalDurationNs'])/tot:6.1f}")
PY
tail -1 gpurun_out/prof_train.log
