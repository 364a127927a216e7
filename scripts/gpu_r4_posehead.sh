#!/bin/bash
# PoseNet heads as one grouped GEMM (nnsx::pw_conv_group): fp64 gates, pose goldens, bench b64 / b512.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_models_f32.py -x -q --timeout 120 --timeout-method thread -k "pw_conv_group or posenet" > gpurun_out/ph_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/ph_pytest.log; exit 1; }
tail -1 gpurun_out/ph_pytest.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pose" > gpurun_out/ph_pytest2.log 2>&1 || { echo "pytest2 failed"; tail -40 gpurun_out/ph_pytest2.log; exit 1; }
tail -1 gpurun_out/ph_pytest2.log
out=gpurun_out/posehead_ab.txt
: > $out
for B in 64 512; do
  timeout -k 10 200 python bench.py --config posenet --batch $B --steps 60 --warmup 10 --sweep "" --latency-frames ${LATF:-0} > gpurun_out/ph_b$B.log 2>&1 || { echo "bench B=$B failed"; tail -20 gpurun_out/ph_b$B.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ph_b$B.log') if l.startswith('{')][-1]); print('posenet b$B', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'), d.get('p50_latency_ms_b1'))" | tee -a $out
done
