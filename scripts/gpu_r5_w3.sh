#!/bin/bash
# pre-split x3 weights: numerics tests, tile sweep, layers, bench
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/w3_tests.txt 2>&1
tail -2 gpurun_out/w3_tests.txt
timeout -k 10 300 python -u scripts/x3_tiles.py > gpurun_out/w3_tiles.txt 2>&1
timeout -k 10 300 python bench.py --sweep "" --latency-frames 0 > gpurun_out/w3_bench.json 2>/dev/null
timeout -k 10 300 python bench.py --config posenet --batch 64 --sweep "" --latency-frames 0 > gpurun_out/w3_posenet.json 2>/dev/null
grep -h -o '"value": [0-9.]*, "unit[^,]*, "n_gpus": 1, "steps": [0-9]*, "warmup": [0-9]*, "ms_per_step": [0-9.]*' gpurun_out/w3_bench.json gpurun_out/w3_posenet.json
