#!/bin/bash
# Everything profiles/<round>/ holds, in one GPU session (after scripts/gpu_round.sh passed):
#   train_step_kernel_stats.csv   rocprofv3 kernel-trace stats of the replayed C2 1vsAll step
#   eval_kernel_stats.csv         the same for the filtered evaluation of the test split
#   pmc_traffic.json              HBM bytes per launch of the headline contraction
#   pmc_step_kernels.txt          issue / stall counters of the step's three MFMA kernels
# Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/profiles
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/train -o run -- \
  python3 $R/scripts/dev/prof_train.py complex 1vsAll > $OUT/train.log 2>&1 || { echo "train profile failed"; tail $OUT/train.log; exit 1; }
cp $(find $OUT/train -name "run_kernel_stats.csv") $OUT/train_step_kernel_stats.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/eval -o run -- \
  python3 $R/scripts/dev/prof_eval.py > $OUT/eval.log 2>&1 || { echo "eval profile failed"; tail $OUT/eval.log; exit 1; }
cp $(find $OUT/eval -name "run_kernel_stats.csv") $OUT/eval_kernel_stats.csv
bash $R/scripts/pmc_traffic.sh > $OUT/pmc_traffic.log 2>&1 || { echo "pmc traffic failed"; tail $OUT/pmc_traffic.log; exit 1; }
cp $R/gpurun_out/pmc_traffic/pmc_traffic.json $OUT/pmc_traffic.json
i=0
for set in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- \
    python3 $R/scripts/dev/prof_train.py complex 1vsAll > /dev/null 2> $OUT/pmc_err$i.txt \
    || { echo "pmc pass $i failed"; tail -3 $OUT/pmc_err$i.txt; exit 1; }
done
cd $R
python3 - "$OUT" > $OUT/pmc_step_kernels.txt <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
kernels = {"forward  score_dot_persist16 (2,048 x 14,541 x 512)": "score_dot_persist16",
           "dQ       bwd3p_q (G planes . E)": "bwd3p_q_kernel",
           "dE       bwd3p_t (G planes^T . Q planes)": "bwd3p_t_kernel"}
vals = {k: collections.defaultdict(list) for k in kernels}
for fn in sorted(glob.glob(f"{root}/pmc*/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(fn)):
        for k, pat in kernels.items():
            if pat in row.get("Kernel_Name", ""):
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
names = sorted({c for v in vals.values() for c in v})
print("rocprofv3 --pmc (kernel-trace only, one pass per counter group) over scripts/dev/prof_train.py:")
print("mean counter value per dispatch of the three MFMA kernels of the replayed C2 1vsAll step\n")
print(f"{'counter':32s}" + "".join(f"{k.split()[0]:>16s}" for k in kernels))
for c in names:
    print(f"{c:32s}" + "".join(f"{(sum(vals[k][c]) / len(vals[k][c]) if vals[k][c] else float('nan')):16.1f}"
                               for k in kernels))
print()
for k in kernels:
    print(k)
PY
cat $OUT/pmc_step_kernels.txt
