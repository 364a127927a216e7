#!/bin/bash
# 5x5 tiles for SSD's 10x10 stage: numerics, then SSD A/B (NNSX_IRW_SKIP=17,18: the 7x7 tiles as before)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ssd5.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pt_ssd5.log; exit 1; }
tail -1 gpurun_out/pt_ssd5.log
for spec in "new:NNSX_NONE=1" "old:NNSX_IRW_SKIP=17,18" "new2:NNSX_NONE=1"; do
  n=${spec%%:*}; e=${spec#*:}
  env $e timeout -k 10 170 python bench.py --config ssd --batch 64 --steps 30 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/ssd5_$n.log 2>&1 || { echo "bench $n failed"; tail -20 gpurun_out/ssd5_$n.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ssd5_$n.log') if l.startswith('{')][-1]); print('ssd $n', d['value'], d['ms_per_step'])"
done
