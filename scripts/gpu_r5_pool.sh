#!/bin/bash
# avgpool with 4-quad workgroups on small grids (HEAD tree) vs variants/base, same box
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_models_f32.py tests/test_gpu_x3.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pool_tests.txt 2>&1
grep -E "passed|failed" gpurun_out/pool_tests.txt
for rep in 1 2 3; do
  for arm in new base; do
    b=bench.py; [ $arm = base ] && b=variants/base/bench.py
    timeout -k 10 300 python $b --config deeplab --batch 8 --sweep "" --latency-frames 0 > gpurun_out/pool.json 2>/dev/null
    echo "$rep $arm deeplab b8 $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/pool.json)"
  done
done
