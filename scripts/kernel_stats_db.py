#!/usr/bin/env python3
"""Per-kernel totals of a rocprofv3 results.db (rocpd sqlite): dispatch count,
total and mean duration, sorted by total.  Optional second argument: divide
totals by this many steps (per-step view).

    python scripts/kernel_stats_db.py gpurun_out/prof_x/x_results.db [steps] [top]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    c = sqlite3.connect(db)
    rows = c.execute("select name, end - start from kernels").fetchall()
    agg = {}
    for n, d in rows:
        n = n.replace("(anonymous namespace)::", "").replace("nnsx::kernels::", "")
        k = (n[5:] if n.startswith("void ") else n).split("(")[0][:110]
        a = agg.setdefault(k, [0, 0])
        a[0] += 1
        a[1] += d
    tot = sum(v[1] for v in agg.values())
    print(f"# {db}: {len(rows)} dispatches, {tot / 1e6:.3f} ms kernel time"
          + (f", per step ({steps:g} steps): {tot / 1e3 / steps:.1f} us" if steps != 1 else ""))
    print(f"{'calls':>7s} {'total us':>10s} {'per step':>9s} {'mean us':>8s}  kernel")
    for k, (n, d) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{n:7d} {d / 1e3:10.1f} {d / 1e3 / steps:9.1f} {d / n / 1e3:8.2f}  {k}")


if __name__ == "__main__":
    main()
