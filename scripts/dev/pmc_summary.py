"""Summarise rocprofv3 --pmc csv passes: mean counter value per dispatch for one kernel."""
import csv, glob, sys, collections
root = sys.argv[1]; pat = sys.argv[2] if len(sys.argv) > 2 else 'score_dot'
vals = collections.defaultdict(list)
for fn in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for row in csv.DictReader(open(fn)):
        if pat in row.get('Kernel_Name', ''):
            vals[row['Counter_Name']].append(float(row['Counter_Value']))
for k, v in sorted(vals.items()):
    print(f"{k:32s} {sum(v)/len(v):16.1f}  (n={len(v)})")
