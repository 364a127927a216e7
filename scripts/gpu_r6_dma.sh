#!/bin/bash
# is the sustained headline bound by the frame upload?  rocprofv3 kernel + memory-copy trace of a 100-step
# bench.py run (device ms per invoke series too), then the copy durations / rates over time.
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6dma}
mkdir -p $O
export TMPDIR=/tmp NNSX_BENCH_SERIES=1
R=$PWD
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/$O/prof -o run --output-format csv -- \
   python3 $R/bench.py --sweep "" --latency-frames 0 > $R/$O/bench.json 2> $R/$O/bench.err)
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench.json | tr '\n' ' '; echo
python3 - $O <<'PY'
import csv, glob, sys, statistics
d = sys.argv[1]
mc = glob.glob(f"{d}/prof/**/*memory_copy_trace.csv", recursive=True)
kt = glob.glob(f"{d}/prof/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(mc[0])))
big = [r for r in rows if int(r.get("Size", r.get("size", 0)) or 0) > 1 << 20]
print(len(rows), "copies,", len(big), "> 1 MB; columns:", list(rows[0])[:12])
def f(r, *ks):
    for k in ks:
        if k in r: return r[k]
out = []
for r in big:
    s, e, n = int(f(r, "Start_Timestamp")), int(f(r, "End_Timestamp")), int(f(r, "Size"))
    out.append((s, e, n))
out.sort()
t0 = out[0][0]
print("first 12 / last 12 large copies: start ms, duration us, MB, GB/s")
for s, e, n in out[:12] + out[-12:]:
    print(f"{(s - t0) / 1e6:9.3f} {(e - s) / 1e3:9.1f} {n / 1e6:7.2f} {n / max(1, e - s):6.2f}")
rates = [n / max(1, e - s) for s, e, n in out]
print("rate GB/s median first 20 / rest:", statistics.median(rates[:20]), statistics.median(rates[20:]) if len(rates) > 20 else None)
PY
grep -h "device ms per invoke" $O/bench.err | cut -c1-500
