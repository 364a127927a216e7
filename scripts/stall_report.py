#!/usr/bin/env python3
"""Per-step GPU busy / idle and stalled kernels out of a rocprofv3 run with
--kernel-trace --hip-trace --memory-copy-trace (csv).

    python scripts/stall_report.py <dir with run_kernel_trace.csv ...> [step-kernel-substring]

A step is the span from one launch of the step's first kernel (default the
fused stem) to the next.  A kernel is reported as stalled when it takes more
than 2.5x its median over the run; for each, the host HIP calls of the other
threads that were in flight across it and the copies around it are listed.
"""
import csv
import os
import re
import statistics
import sys
from collections import defaultdict

root = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "stem_ir1w"


def load(name):
    p = os.path.join(root, name)
    return list(csv.DictReader(open(p))) if os.path.exists(p) else []


def short(n):
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:60]


ks = load("run_kernel_trace.csv")
ks.sort(key=lambda r: int(r["Start_Timestamp"]))
api = load("run_hip_api_trace.csv")
mc = load("run_memory_copy_trace.csv")
for r in ks:
    r["s"], r["e"], r["n"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])

starts = [i for i, r in enumerate(ks) if first in r["Kernel_Name"]]
print(f"{len(starts)} launches of {first}")
print(f"{'step':>4} {'span us':>9} {'busy us':>9} {'idle us':>8} kernels")
for k in range(len(starts) - 1):
    seg = ks[starts[k]:starts[k + 1]]
    t0, t1 = seg[0]["s"], ks[starts[k + 1]]["s"]
    busy, end = 0, t0
    for r in seg:
        busy += min(r["e"], t1) - max(r["s"], end) if r["e"] > end else 0
        end = max(end, r["e"])
    print(f"{k:4d} {(t1 - t0) / 1e3:9.1f} {busy / 1e3:9.1f} {(t1 - t0 - busy) / 1e3:8.1f} {len(seg)}")

dur = defaultdict(list)
for r in ks:
    dur[r["n"]].append(r["e"] - r["s"])
med = {n: statistics.median(v) for n, v in dur.items()}
slow = [r for r in ks if len(dur[r["n"]]) >= 4 and r["e"] - r["s"] > 2.5 * med[r["n"]] and r["e"] - r["s"] > 100e3]
print(f"\n{len(slow)} stalled kernels (> 2.5x their median, > 100 us)")
skip = {"hipGetDevice", "hipSetDevice", "hipGetLastError", "hipStreamGetCaptureInfo", "__hipPushCallConfiguration",
        "__hipPopCallConfiguration"}
for r in slow:
    s, e = r["s"], r["e"]
    print(f"- {r['n']}: {(e - s) / 1e3:.1f} us (median {med[r['n']] / 1e3:.1f} us)")
    for a in api:
        a0, a1 = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
        if a["Function"] in skip or a1 - a0 < 1e6 or a1 < s or a0 > e:
            continue
        print(f"    host tid {a['Thread_Id']} {a['Function']}: {(a0 - s) / 1e3:+.1f} .. {(a1 - s) / 1e3:+.1f} us")
    for m in mc:
        m0, m1 = int(m["Start_Timestamp"]), int(m["End_Timestamp"])
        if m1 > s - 3e6 and m0 < e + 3e6:
            print(f"    copy {m['Direction'].replace('MEMORY_COPY_', '')}: {(m0 - s) / 1e3:+.1f} us, {(m1 - m0) / 1e3:.1f} us")
