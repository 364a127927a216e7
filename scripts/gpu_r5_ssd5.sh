#!/bin/bash
# SSD's 19x19 blocks on 5x5 tiles (least-padding pick) vs 7x7 (NNSX_IRW_SKIP=22,23,24 drops the 5x5 configurations)
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/ssd5_tests.txt 2>&1
tail -1 gpurun_out/ssd5_tests.txt
for rep in 1 2; do
  for arm in t5 t7; do
    if [ $arm = t7 ]; then export NNSX_IRW_SKIP=22,23,24; else unset NNSX_IRW_SKIP; fi
    timeout -k 10 300 python bench.py --config ssd --batch 64 --sweep "" --latency-frames 0 > gpurun_out/ssd5_$arm.json 2>/dev/null
    echo "$rep $arm $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ssd5_$arm.json)"
  done
done
