#!/bin/bash
# PMC passes (kernel-trace only) over scripts/dev/dist_one.py (or dist_bwd_one.py): usage pmc_dist.sh [kind] [script]
set -o pipefail
mkdir -p gpurun_out/pmcd
export TMPDIR=/tmp
K=${1:-0}
SCRIPT=${2:-dist_one.py}
cd /tmp
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmcd/p$i -o run -- python3 $GRAFT_REPO_ROOT/scripts/dev/$SCRIPT $K 2 > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/pmcd/err$i.txt || { echo "pass $i failed"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/pmcd/err$i.txt; exit 1; }
done
cd $GRAFT_REPO_ROOT
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(list)
for fn in glob.glob("gpurun_out/pmcd/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if "dist" in r["Kernel_Name"]:
            tot[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(tot.items()):
    print(f"{k:60s} {c:28s} mean/dispatch {sum(v)/len(v):.4g}  (n={len(v)})")
PY
