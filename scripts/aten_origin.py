"""Where do the ATen kernels of a bench run come from?  (round-3 verdict: ~1.8k
reduce_kernel / vectorized_elementwise_kernel dispatches per run, origin unknown)

usage: python scripts/aten_origin.py <results.db>

For every stream: dispatch counts of ATen kernels (at::native / reduce_kernel /
vectorized_elementwise) vs nnsx kernels, and whether the ATen dispatches fall
inside the window of the filter's timed forwards (between the first and last
nnsx model kernel of the busiest nnsx stream) or outside it (model load,
freeze / constant folding, capture warm-up).
"""
import sqlite3
import sys


def is_aten(n):
    if "nnsx" in n:  # (irw_reduce_kernel etc.)
        return False
    return "at::native" in n or n.startswith("void at::") or "reduce_kernel" in n or "elementwise_kernel" in n


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, stream_id, start, end from kernels order by start").fetchall()
    streams = {}
    for name, sid, st, en in rows:
        d = streams.setdefault(sid, {"aten": 0, "nnsx": 0, "other": 0, "first": None, "last": None})
        if is_aten(name):
            d["aten"] += 1
        elif "nnsx" in name or "irw_" in name or "stem_" in name or "pw_" in name:
            d["nnsx"] += 1
            d["first"] = st if d["first"] is None else d["first"]
            d["last"] = en
        else:
            d["other"] += 1
    busiest = max(streams, key=lambda s: streams[s]["nnsx"])
    t0, t1 = streams[busiest]["first"], streams[busiest]["last"]
    print(f"# {db}: {len(rows)} dispatches; busiest nnsx stream {busiest} ({streams[busiest]['nnsx']} nnsx kernels)")
    for sid, d in sorted(streams.items()):
        print(f"stream {sid}: aten {d['aten']}, nnsx {d['nnsx']}, other {d['other']}")
    inside = [r for r in rows if is_aten(r[0]) and t0 <= r[2] <= t1]
    outside = [r for r in rows if is_aten(r[0]) and not (t0 <= r[2] <= t1)]
    print(f"ATen dispatches inside the forward window: {len(inside)}, outside: {len(outside)}")
    by = {}
    for n, sid, st, en in inside:
        by.setdefault((n.split("(")[0][:90], sid), []).append(en - st)
    for (n, sid), v in sorted(by.items(), key=lambda kv: -len(kv[1]))[:15]:
        print(f"  inside  stream {sid}: {len(v):6d} x {sum(v) / len(v) / 1000:7.1f} us  {n}")
    # bursts: ATen dispatches grouped by gaps > 5 ms (load / capture phases)
    bursts, cur = [], []
    for r in [r for r in rows if is_aten(r[0])]:
        if cur and r[2] - cur[-1][3] > 5_000_000:
            bursts.append(cur)
            cur = []
        cur.append(r)
    if cur:
        bursts.append(cur)
    print(f"ATen bursts (gap > 5 ms): {len(bursts)}")
    for b in bursts[:20]:
        print(f"  t={(b[0][2] - rows[0][2]) / 1e6:9.1f} ms  {len(b):5d} dispatches over {(b[-1][3] - b[0][2]) / 1e6:8.1f} ms"
              f"  streams {sorted(set(r[1] for r in b))}")


if __name__ == "__main__":
    main(sys.argv[1])
