#!/bin/bash
# host time of tensor_filter's hipGraphLaunch in the headline pipeline under runtime variants:
# rocprofv3 --hip-runtime-trace of a 30-step bench.py run per variant, median hipGraphLaunch us.
#   scripts/gpu_r6_launch.sh <outdir> "<variant>" ...
set -eo pipefail
cd "$(dirname "$0")/.."
O=$1; shift
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
for v in "$@"; do
  tag=$(echo "$v" | tr ' =' '__')
  (cd /tmp && env $v timeout -k 10 300 rocprofv3 --hip-runtime-trace -d $R/$O/$tag -o run --output-format csv -- \
     python3 $R/bench.py --sweep "" --latency-frames 0 --steps 30 --warmup 10 > $R/$O/$tag.json 2> $R/$O/$tag.err)
  python3 - "$O/$tag" "$v" <<'PY'
import csv, glob, statistics, sys
f = glob.glob(sys.argv[1] + "/**/*hip_api_trace.csv", recursive=True)[0]
g = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f)) if r["Function"] == "hipGraphLaunch")
d = [(e - s) / 1e3 for s, e in g]
print(f"[{sys.argv[2]}] {len(d)} hipGraphLaunch, median {statistics.median(d[5:]):.1f} us, min {min(d[5:]):.1f}, max {max(d[5:]):.1f}")
PY
  grep -o '"value": [0-9.]*' $O/$tag.json || true
  rm -rf $O/$tag
done
