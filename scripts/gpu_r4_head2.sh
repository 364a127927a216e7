#!/bin/bash
# headline bench twice (run-to-run spread on one box)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 170 python bench.py --sweep "" --latency-frames 0 > gpurun_out/head2_$i.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/head2_$i.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/head2_$i.log') if l.startswith('{')][-1]); print('mbv2 b512 run $i', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))"
done
