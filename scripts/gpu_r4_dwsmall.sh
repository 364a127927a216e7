#!/bin/bash
# depthwise multi-pixel lanes only on large maps: gates + batch-1 latency of the configs
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dw_conv or models_f32" > gpurun_out/dws_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/dws_pytest.log; exit 1; }
tail -1 gpurun_out/dws_pytest.log
for spec in posenet:64 deeplab:8 ssd:64; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 170 python bench.py --config $c --batch $B --steps 30 --warmup 10 --sweep "" > gpurun_out/dws_${c}.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/dws_${c}.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dws_${c}.log') if l.startswith('{')][-1]); print('$c b$B', d['value'], d['ms_per_step'], d.get('p50_latency_ms'), d.get('p50_latency_ms_b1'), d.get('p99_latency_ms_b1'))"
done
