#!/bin/bash
# XE defaults + DeepLab batch-1 changes: tests, DeepLab b1 kernel trace, same-box A/B vs variants/base
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 900 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/xe2_tests.txt 2>&1
tail -2 gpurun_out/xe2_tests.txt

SPECS="mbv2:512 deeplab:1 deeplab:8 ssd:64 posenet:64" bash scripts/gpu_ab_variant.sh
