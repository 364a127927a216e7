#!/bin/bash
# pipelined x3 GEMM: tests, tile sweeps (new / base), same-box bench A/B
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/pp_tests.txt 2>&1
tail -2 gpurun_out/pp_tests.txt
timeout -k 10 300 python -u scripts/x3_tiles.py > gpurun_out/pp_tiles_new.txt 2>&1
timeout -k 10 300 python -u variants/base/scripts/x3_tiles.py > gpurun_out/pp_tiles_base.txt 2>&1
SPECS="mbv2:512 posenet:64 deeplab:8 ssd:64" bash scripts/gpu_ab_variant.sh
