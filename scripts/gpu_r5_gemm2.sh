#!/bin/bash
# x3 GEMM v2 (own unit with VGPR-form MFMA, pre-split weights, conflict-free planes, x3 tile pick)
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/g2_tests.txt 2>&1
tail -2 gpurun_out/g2_tests.txt
timeout -k 10 300 python -u scripts/x3_tiles.py > gpurun_out/g2_tiles.txt 2>&1
for spec in mbv2:512 posenet:64 ssd:64 deeplab:8; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --batch $B --sweep "" --latency-frames 0 > gpurun_out/g2_$c.json 2>/dev/null
  grep -h -o '"value": [0-9.]*, "unit[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/g2_$c.json
done
SPECS="25088,960,320,x3,128064 18496,1024,1024,x3,64064" bash scripts/gpu_r5_pmc_gemm.sh > gpurun_out/g2_pmc.txt 2>&1
cat gpurun_out/g2_pmc.txt
