#!/bin/bash
# x3 GEMM tile rule by grid fill (HEAD tree) vs variants/base (the previous rule), same box;
# DeepLab's 33x33 blocks on 5 x 5 tiles (NNSX_IRW_SKIP=7,8,9 drops the 7 x 7 configurations)
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_x3.py -q -x --timeout 300 --timeout-method thread > gpurun_out/fill_tests.txt 2>&1
tail -1 gpurun_out/fill_tests.txt
for rep in 1 2; do
  for spec in deeplab:8 ssd:64 posenet:64 mbv2:512; do
    c=${spec%%:*}; B=${spec##*:}
    for arm in new base; do
      if [ $arm = new ]; then b=bench.py; else b=variants/base/bench.py; fi
      timeout -k 10 300 python $b --config $c --batch $B --sweep "" --latency-frames 0 > gpurun_out/fill_${arm}_$c.json 2>/dev/null
      echo "$rep $arm $c $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/fill_${arm}_$c.json)"
    done
  done
  NNSX_IRW_SKIP=7,8,9 timeout -k 10 300 python bench.py --config deeplab --batch 8 --sweep "" --latency-frames 0 > gpurun_out/fill_t5_deeplab.json 2>/dev/null
  echo "$rep new-t5 deeplab $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/fill_t5_deeplab.json)"
done
