#!/bin/bash
# batch-1 live-camera latency of configs 3-5 vs camera rate
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in deeplab:30 deeplab:100 deeplab:250 posenet:100 posenet:250 posenet:500 ssd:500; do
  c=${spec%%:*}; f=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --batch 8 --steps 5 --warmup 2 --sweep "" --latency-fps $f --latency-frames 200 > gpurun_out/lat_${c}_$f.log 2>&1 || { echo "lat $spec failed"; tail -20 gpurun_out/lat_${c}_$f.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/lat_${c}_$f.log') if l.startswith('{')][-1]); print('$c fps=$f', d.get('p50_latency_ms_b1'), d.get('p99_latency_ms_b1'))"
done
