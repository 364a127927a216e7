"""Per-dispatch listing of the last forward on the busiest non-load stream of a rocprofv3 results.db:
us, grid, kernel.  usage: python scripts/fwd_trace.py <results.db> <first-kernel-substring> [stream]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
first = sys.argv[2]
if len(sys.argv) > 3:
    st = int(sys.argv[3])
else:
    st = c.execute(f"select stream_id from kernels where name like '%{first}%' group by stream_id "
                   "order by count(*) desc limit 1").fetchone()[0]
rows = c.execute("select name, end-start, grid_x, grid_y, workgroup_x from kernels where stream_id=? order by start",
                 (st,)).fetchall()
idx = [i for i, r in enumerate(rows) if first in r[0]]
f = rows[idx[-1]:]
tot = 0.0
for n, d, gx, gy, w in f:
    n = n.replace("(anonymous namespace)::", "").replace("nnsx::kernels::", "")
    n = (n[5:] if n.startswith("void ") else n).split("(")[0]
    tot += d / 1e3
    print(f"{d / 1e3:8.1f} us  grid {gx // max(w, 1):6d} x {gy:4d}  {n[:90]}")
print(f"# stream {st}: {len(f)} dispatches, {tot:.1f} us")
