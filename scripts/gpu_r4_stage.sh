#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_stage.py tests/test_gpu_models_f32.py tests/test_gpu_elements.py tests/test_gpu_decoders_golden.py tests/test_gpu_pipelines.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_stage.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_stage.log; exit 1; }
tail -3 gpurun_out/pytest_stage.log
bash scripts/gpu_r4_configs.sh
