#!/bin/bash
# odd-map tiles (HEAD tree) vs variants/base, same box: 11 x 5 on DeepLab's 33x33 (kIrwCfgs 28-30),
# 5 x 10 / 5 x 13 on 32 -> 192 -> 32 (31 / 32), 5 x 15 on 24 -> 144 -> 24 (33); arms drop one family each
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_x3.py -q -x --timeout 300 --timeout-method thread -k "ir_block or model" > gpurun_out/tiles2_tests.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread >> gpurun_out/tiles2_tests.txt 2>&1
grep -E "passed|failed" gpurun_out/tiles2_tests.txt
run() {  # arm skip config batch
  local b=bench.py; [ $1 = base ] && b=variants/base/bench.py
  NNSX_IRW_SKIP=$2 timeout -k 10 300 python $b --config $3 --batch $4 --sweep "" --latency-frames 0 > gpurun_out/tiles2.json 2>/dev/null
  echo "$rep $1 $3 b$4 $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/tiles2.json)"
}
for rep in 1 2; do
  for cb in ssd:64 deeplab:8; do
    c=${cb%%:*}; B=${cb##*:}
    run new "" $c $B; run base "" $c $B; run no11x5 28,29,30 $c $B; run no5x13 32 $c $B; run no5x15 33 $c $B
  done
done
