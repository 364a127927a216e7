#!/bin/bash
# Round 4 final check: whole GPU suite, smoke, default bench, the three single-GPU configs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_final.log; exit 1; }
tail -2 gpurun_out/pytest_final.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 170 python bench.py > gpurun_out/bench_final.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-400
for spec in posenet:64 ssd:64 deeplab:8 deeplab:32; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 170 python bench.py --config $c --batch $B --steps 30 --warmup 10 --sweep "" > gpurun_out/final_${c}_b$B.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/final_${c}_b$B.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/final_${c}_b$B.log') if l.startswith('{')][-1]); print('$c b$B', d['value'], d['ms_per_step'], d.get('p50_latency_ms'), d.get('p50_latency_ms_b1'), d.get('p99_latency_ms_b1'))"
done
