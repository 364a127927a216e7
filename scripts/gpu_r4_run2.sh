#!/bin/bash
# Round 4, second pass: decoder numerics after the pose raster change, then the
# model configs with the dwpw fusions off (defaults) and a PoseNet trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_decoders_golden.py tests/test_gpu_decode_stage.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_run2.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_run2.log; exit 1; }
tail -2 gpurun_out/pytest_run2.log
SPECS="ssd:64 deeplab:8 deeplab:16 deeplab:32 posenet:64" TRACES="posenet:64 ssd:64" bash scripts/gpu_r4_configs.sh
