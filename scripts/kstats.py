"""Summarise a rocprofv3 output directory: kernels by total time (calls, total
ms, average us, share), names shortened.

    python scripts/kstats.py <rocprof -d dir> [--top N] [--window] [--per-step K]

Default: the run's kernel_stats.csv (every kernel of the process: model export,
warm-up and checks included).  --window (needs --kernel-trace and
--marker-trace): only the kernels that STARTED between the two roctx marks
bench.py's tensor_sink emits at the arrivals of batch W and batch W + K
("nnsx:<sink>:<count>", tensor_sink roctx-marks) -- the timed region's own
kernels; --per-step K divides the totals by the K timed steps.
"""
import argparse
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    name = name.replace("nnsx::kernels::(anonymous namespace)::", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\((?!anonymous).*", "", name).replace("void ", "")


def find(d, pattern):
    f = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return f[0] if f else None


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(f"none of {names} in {list(row)}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--window", action="store_true")
    ap.add_argument("--per-step", type=int, default=0)
    a = ap.parse_args()
    if not a.window:
        f = find(a.dir, "*kernel_stats.csv")
        if not f:
            sys.exit(f"no kernel_stats.csv under {a.dir}")
        rows = [(short(r["Name"]), int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(f))]
        src = f
    else:
        kf, mf = find(a.dir, "*kernel_trace.csv"), find(a.dir, "*marker_api_trace.csv")
        if not kf or not mf:
            sys.exit(f"--window needs kernel_trace.csv and marker_api_trace.csv under {a.dir}")
        marks = []
        for r in csv.DictReader(open(mf)):
            text = " ".join(str(v) for v in r.values())
            m = re.search(r"nnsx:[^:\s]+:(\d+)", text)
            if m:
                marks.append((int(col(r, "Start_Timestamp", "start_timestamp")), int(m.group(1))))
        marks.sort()
        if len(marks) < 2:
            sys.exit(f"found {len(marks)} nnsx roctx marks in {mf} (need the window's two)")
        (t0, n0), (t1, n1) = marks[0], marks[-1]
        agg = defaultdict(lambda: [0, 0.0])
        for r in csv.DictReader(open(kf)):
            s0 = int(col(r, "Start_Timestamp", "start_timestamp"))
            s1 = int(col(r, "End_Timestamp", "end_timestamp"))
            if t0 <= s0 < t1:
                e = agg[short(col(r, "Kernel_Name", "kernel_name", "Name"))]
                e[0] += 1
                e[1] += s1 - s0
        rows = [(k, v[0], v[1]) for k, v in agg.items()]
        src = f"{kf}, window between marks at buffers {n0} and {n1} ({(t1 - t0) / 1e6:.3f} ms)"
    total = sum(r[2] for r in rows)
    rows.sort(key=lambda r: -r[2])
    k = a.per_step or 1
    print(f"# {src}: {total / 1e6:.3f} ms of kernels" + (f", {total / 1e6 / k:.4f} ms per step ({k} steps)" if a.per_step else ""))
    unit = "per step" if a.per_step else "total"
    print(f"{'calls':>7} {'ms ' + unit:>14} {'avg us':>8} {'%':>6}  kernel")
    for name, calls, ns in rows[:a.top]:
        print(f"{calls / k:7.1f} {ns / 1e6 / k:14.4f} {ns / calls / 1e3:8.1f} {100 * ns / total:6.1f}  {name[:110]}")


if __name__ == "__main__":
    main()
