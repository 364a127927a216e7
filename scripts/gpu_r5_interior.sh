#!/bin/bash
# wave-uniform interior-tile fast paths (HEAD tree) vs variants/base, same box
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_x3.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/interior_tests.txt 2>&1
grep -E "passed|failed" gpurun_out/interior_tests.txt
for rep in 1 2 3; do
  for spec in mbv2:512 ssd:64 deeplab:8; do
    c=${spec%%:*}; B=${spec##*:}
    for arm in new base; do
      b=bench.py; [ $arm = base ] && b=variants/base/bench.py
      timeout -k 10 300 python $b --config $c --batch $B --sweep "" --latency-frames 0 > gpurun_out/interior.json 2>/dev/null
      echo "$rep $arm $c b$B $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/interior.json)"
    done
  done
done
