#!/bin/bash
# stem staging change: gates, PoseNet bench, per-kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "stem or posenet or pose" > gpurun_out/stem_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/stem_pytest.log; exit 1; }
tail -1 gpurun_out/stem_pytest.log
for B in 64 512; do
  timeout -k 10 170 python bench.py --config posenet --batch $B --steps 40 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/stem_b$B.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/stem_b$B.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/stem_b$B.log') if l.startswith('{')][-1]); print('posenet b$B', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))"
done
