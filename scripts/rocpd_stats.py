"""Kernel statistics from a rocprofv3 SQLite output (`<name>_results.db`).

usage: python scripts/rocpd_stats.py <results.db> [top] [--stream N]

Prints per-kernel totals (time, calls, average) sorted by total time, and the
share of each kernel in the summed kernel time.  --stream restricts the table
to one HIP stream (the filter's compute stream holds the timed forwards; the
load-time ATen work of torch.jit.load runs on stream 0).
"""
import sqlite3
import sys


def main(argv):
    db = argv[0]
    top = int(argv[1]) if len(argv) > 1 and not argv[1].startswith("--") else 30
    stream = None
    if "--stream" in argv:
        stream = int(argv[argv.index("--stream") + 1])
    c = sqlite3.connect(db)
    where = f"where stream_id = {stream}" if stream is not None else ""
    rows = c.execute(f"select name, count(*), sum(end - start) / 1000.0, avg(end - start) / 1000.0 "
                     f"from kernels {where} group by name order by 3 desc").fetchall()
    total = sum(r[2] for r in rows) or 1.0
    print(f"# {db}{'' if stream is None else f' (stream {stream})'}: {len(rows)} kernels, "
          f"{sum(r[1] for r in rows)} dispatches, {total:.1f} us summed")
    print(f"{'total us':>12} {'share':>6} {'calls':>7} {'avg us':>9}  kernel")
    for name, n, tot, avg in rows[:top]:
        short = name.replace("nnsx::kernels::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        print(f"{tot:12.1f} {100 * tot / total:5.1f}% {n:7d} {avg:9.1f}  {short[:110]}")


if __name__ == "__main__":
    main(sys.argv[1:])
