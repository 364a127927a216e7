#!/bin/bash
# three hidden parts where they balance the waves (HEAD tree) vs variants/base, and variants/n510 (the same
# + native 5 x 10 32-channel blocks instead of their x3 twins), same box
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_x3.py -q -x --timeout 300 --timeout-method thread -k "ir_block" > gpurun_out/parts3_tests.txt 2>&1
grep -E "passed|failed" gpurun_out/parts3_tests.txt
for rep in 1 2; do
  for arm in new base n510; do
    b=bench.py; [ $arm != new ] && b=variants/$arm/bench.py
    timeout -k 10 300 python $b --config deeplab --batch 8 --sweep "" --latency-frames 0 > gpurun_out/parts3.json 2>/dev/null
    echo "$rep $arm deeplab b8 $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/parts3.json)"
    timeout -k 10 300 python $b --steps 20 --latency-frames 0 > gpurun_out/parts3.json 2>/dev/null
    echo "$rep $arm mbv2 sweep $(grep -h -o '"sweep": .*\]' gpurun_out/parts3.json | cut -c1-220)"
    timeout -k 10 300 python $b --config ssd --batch 64 --sweep "" --latency-frames 0 > gpurun_out/parts3.json 2>/dev/null
    echo "$rep $arm ssd b64 $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/parts3.json)"
  done
done
