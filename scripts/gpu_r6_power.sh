#!/bin/bash
# sustained-load A/B: per-invoke device ms (NNSX_BENCH_SERIES=1) of bench.py's default pipeline over
# 20 + 200 invokes for each variant; reports the median of the first 20 invokes (before the board
# power limit engages) and of invokes 60.. (sustained), plus the bench value.
#   scripts/gpu_r6_power.sh <out file> "<variant>" ...
set -eo pipefail
cd "$(dirname "$0")/.."
out=$1; shift
mkdir -p "$(dirname "$out")"
export NNSX_BENCH_SERIES=1
for v in "$@"; do
  env $v timeout -k 10 300 python bench.py --sweep "" --latency-frames 0 --steps 200 --warmup 20 > /tmp/pw.json 2> /tmp/pw.err
  python3 - "$v" >> "$out" <<'PY'
import json, re, statistics, sys
err = open("/tmp/pw.err").read()
m = re.search(r"device ms per invoke ([0-9. ]+)", err)
s = [float(x) for x in m.group(1).split()] if m else []
j = json.loads([l for l in open("/tmp/pw.json").read().splitlines() if l.startswith("{")][-1])
first = statistics.median(s[1:21]) if len(s) > 21 else 0
sus = statistics.median(s[60:]) if len(s) > 61 else 0
print(f"[{sys.argv[1]}] value {j['value']} ms/step {j['ms_per_step']} | device ms: first 20 {first:.3f}, sustained {sus:.3f}")
PY
  tail -1 "$out"
done
