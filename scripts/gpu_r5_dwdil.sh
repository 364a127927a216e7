#!/bin/bash
# dilated depthwise on residue-grid lanes (HEAD tree) vs variants/base (contiguous 4 x 4 lanes / per-pixel lanes), same box
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -q -x --timeout 300 --timeout-method thread -k "dw_conv or ir_block or model" > gpurun_out/dwdil_tests.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread -k ssd >> gpurun_out/dwdil_tests.txt 2>&1
tail -1 gpurun_out/dwdil_tests.txt
for arm in new base; do
  if [ $arm = new ]; then d=.; else d=variants/base; fi
  echo "== $arm"; timeout -k 10 120 python -u $d/scripts/dw_dil.py
done
for rep in 1 2; do
  for B in 8 1; do
    for arm in new base; do
      if [ $arm = new ]; then b=bench.py; else b=variants/base/bench.py; fi
      timeout -k 10 300 python $b --config deeplab --batch $B --sweep "" --latency-frames 0 > gpurun_out/dwdil_${arm}.json 2>/dev/null
      echo "$rep $arm deeplab b$B $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/dwdil_${arm}.json)"
    done
  done
done
# SSD's 19x19 blocks on 5 x 10 tiles (HEAD tree) vs 5 x 5 (variants/base)
for rep in 1 2; do
  for arm in new base; do
    if [ $arm = new ]; then b=bench.py; else b=variants/base/bench.py; fi
    timeout -k 10 300 python $b --config ssd --batch 64 --sweep "" --latency-frames 0 > gpurun_out/dwdil_ssd_${arm}.json 2>/dev/null
    echo "$rep $arm ssd b64 $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/dwdil_ssd_${arm}.json)"
  done
done
