"""Summarize rocprofv3 --pmc counter_collection.csv files: mean per dispatch per kernel."""
import csv, glob, os, sys
from collections import defaultdict
root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(lambda: defaultdict(float))
    for row in csv.DictReader(open(f)):
        per[(row["Kernel_Name"][:60], row["Dispatch_Id"])][row["Counter_Name"]] += float(row["Counter_Value"])
    for (k, d), cs in per.items():
        for c, v in cs.items():
            vals[k][c].append(v)
for k, cs in vals.items():
    print(k)
    for c, v in sorted(cs.items()):
        print(f"  {c:24s} {sum(v)/len(v):.6g}  (n={len(v)})")
