"""Sum rocprofv3 --pmc counter CSVs per kernel (matching a name substring)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
tot = defaultdict(float)
n = defaultdict(int)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if pat in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k:32s} {tot[k]:16.0f}  (records {n[k]})")
