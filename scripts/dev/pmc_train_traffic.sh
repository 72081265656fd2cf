#!/bin/bash
# HBM traffic per dispatch of the replayed C2 1vsAll step's kernels: separate --pmc passes
# (kernel-trace only) over scripts/dev/prof_train.py; FETCH_SIZE x2 for the 16-B-per-lane reads
# (MI355X_MICROARCH.md HBM section), in MB.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_train
mkdir -p $OUT
cd /tmp
i=0
for ctr in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 $R/scripts/dev/prof_train.py complex 1vsAll > /dev/null 2> $OUT/err$i.txt || { echo "pass $ctr failed"; tail -3 $OUT/err$i.txt; exit 1; }
done
cd $R
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for fn in sorted(glob.glob(f"{root}/p*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(fn)):
        vals[row["Kernel_Name"][:70]][row["Counter_Name"]].append(float(row["Counter_Value"]))
print(f"{'kernel':72s} {'dispatches':>10s} {'read MB (2 x FETCH_SIZE)':>26s} {'write MB':>10s}")
for k, v in sorted(vals.items(), key=lambda kv: -sum(kv[1].get("FETCH_SIZE", [0]))):
    f = v.get("FETCH_SIZE", [0.0]); w = v.get("WRITE_SIZE", [0.0])
    print(f"{k:72s} {len(f):10d} {2 * sum(f) / len(f) * 1024 / 1e6:26.1f} {sum(w) / len(w) * 1024 / 1e6:10.1f}")
PY
