#!/bin/bash
# DeepLab's dilated blocks fused at batch <= 2: tests, then b1 / b2 / b8 A/B (NNSX_IRW_SKIP=22,23,24 = unfused)
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread -k "dilated or deeplab or ir_block or pool_proj" > gpurun_out/dl_tests.txt 2>&1
tail -2 gpurun_out/dl_tests.txt
for rep in 1 2; do
for B in 1 8; do
  for arm in fused unfused; do
    if [ $arm = unfused ]; then export NNSX_IRW_SKIP=22,23,24; else unset NNSX_IRW_SKIP; fi
    timeout -k 10 300 python bench.py --config deeplab --batch $B --steps 200 --warmup 20 --sweep "" > gpurun_out/dl_${arm}_b$B.json 2>/dev/null
    echo "$rep b$B $arm $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/dl_${arm}_b$B.json) $(grep -h -o '"p50_latency_ms": [0-9.]*' gpurun_out/dl_${arm}_b$B.json)"
  done
done
done
export TMPDIR=/tmp
R=$PWD
unset NNSX_IRW_SKIP
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/dl_b1b -o run --output-format csv -- python3 $R/bench.py --config deeplab --batch 1 --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/gpurun_out/dl_b1b.log 2>&1)
echo traced
