#!/usr/bin/env python3
"""Kernel-time summary of a rocprofv3 --kernel-trace run of bench.py: the
kernels of the last full model step (between the last two launches of the
most frequent first-of-step kernel, found as the kernel launched once per
step with the largest grid), plus per-kernel totals over the run.

    python scripts/config_trace_report.py <rocprofv3 output dir>
"""
import collections
import csv
import glob
import os
import re
import sys


def short(n):
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:70]


def main():
    root = sys.argv[1]
    rows = []
    for f in glob.glob(os.path.join(root, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    for r in rows:
        r["s"], r["e"], r["n"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])
    # the step marker: a stem kernel of the fused models
    marks = [i for i, r in enumerate(rows) if re.search(r"stem", r["n"])]
    print(f"# {len(rows)} kernel dispatches; {len(marks)} stem launches")
    if len(marks) >= 3:
        a, b = marks[-3], marks[-2]
        t0 = rows[a]["s"]
        busy = sum(r["e"] - r["s"] for r in rows[a:b])
        print(f"# one step: {(rows[b]['s'] - t0) / 1e3:.1f} us span, {busy / 1e3:.1f} us kernel time, {b - a} kernels")
        for r in rows[a:b]:
            print(f"{(r['s'] - t0) / 1e3:9.1f} us {(r['e'] - r['s']) / 1e3:8.1f} us  {r['n']}  grid={r.get('Grid_Size_X', '')}")
    tot = collections.defaultdict(lambda: [0, 0])
    for r in rows:
        tot[r["n"]][0] += 1
        tot[r["n"]][1] += r["e"] - r["s"]
    print("\n# totals over the run (count, total us, mean us)")
    for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:25]:
        print(f"{c:6d} {t / 1e3:10.1f} {t / 1e3 / c:8.1f}  {n}")


if __name__ == "__main__":
    main()
