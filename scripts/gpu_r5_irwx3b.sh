#!/bin/bash
# new x3 twin defaults: tests, then same-box A/B vs variants/base
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/ixb_tests.txt 2>&1
tail -2 gpurun_out/ixb_tests.txt
SPECS="mbv2:512 ssd:64 deeplab:8" bash scripts/gpu_ab_variant.sh
