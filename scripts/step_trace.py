"""One model step out of a rocprofv3 kernel trace: the kernels between the last
two launches of the stem kernel, in launch order, with their durations.

usage: python scripts/step_trace.py <rocprofv3 output dir> [stem-substring]
"""
import csv
import glob
import os
import re
import sys

root = sys.argv[1]
stem = sys.argv[2] if len(sys.argv) > 2 else "stem_mfma_kernel"
rows = []
for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if stem in r["Kernel_Name"]]
if len(starts) < 3:
    sys.exit("fewer than 3 steps in the trace")
a, b = starts[-3], starts[-2]
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
total = 0
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    total += d
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("nnsx::kernels::", "")
    name = re.sub(r"\(.*", "", name[5:] if name.startswith("void ") else name)
    g = r.get("Grid_Size_X", r.get("Grid_Size", ""))
    print(f"{(int(r['Start_Timestamp']) - t0) / 1000:9.1f} us  {d:8.1f} us  grid {g:>8}  {name[:90]}")
span = (int(rows[b]["Start_Timestamp"]) - t0) / 1000
print(f"kernels {len(step)}  busy {total:.1f} us  step span {span:.1f} us")
