#!/bin/bash
# SSD heads: grouped depthwise + grouped GEMM (sep_heads mode 0, default) vs 2 launches per head
# (NNSX_SSD_SEP_HEADS=0): fp64 gates, then bench.py --config ssd at batch 64 and 512.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_models_f32.py -x -q --timeout 120 --timeout-method thread -k "sep_heads or ssd" > gpurun_out/heads_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/heads_pytest.log; exit 1; }
tail -1 gpurun_out/heads_pytest.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ssd or bbox or bounding" > gpurun_out/heads_pytest2.log 2>&1 || { echo "pytest2 failed"; tail -40 gpurun_out/heads_pytest2.log; exit 1; }
tail -1 gpurun_out/heads_pytest2.log
out=gpurun_out/heads_ab.txt
: > $out
for B in 64 512; do
  for v in 1 0 1 0; do
    NNSX_SSD_SEP_HEADS=$v timeout -k 10 200 python bench.py --config ssd --batch $B --steps ${STEPS:-60} --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/heads_b${B}_$v.log 2>&1 || { echo "bench B=$B v=$v failed"; tail -20 gpurun_out/heads_b${B}_$v.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/heads_b${B}_$v.log') if l.startswith('{')][-1]); print('ssd b$B grouped_heads=$v', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))" | tee -a $out
  done
done
