#!/bin/bash
# expand-x3 (XE) twins of the native fused blocks: accuracy tests and per-block A/B with NNSX_X3_IRW=2;
# then the DeepLab batch-1 script
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
NNSX_X3_IRW=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py -q --timeout 300 --timeout-method thread -k "ir_block" > gpurun_out/xe_tests.txt 2>&1 || true
grep -E "FAILED|passed|failed" gpurun_out/xe_tests.txt | tail -12
NNSX_X3_IRW=2 timeout -k 10 400 python -u scripts/x3_blocks_ab.py 512 3 > gpurun_out/xe_blocks_ab.txt 2>&1
cat gpurun_out/xe_blocks_ab.txt
bash scripts/gpu_r5_dlb1.sh
