#!/bin/bash
# irw_x3 in its own VGPR-form unit: x3 tests with every twin on, per-block A/B, bench
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
NNSX_X3_IRW=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py -q --timeout 300 --timeout-method thread > gpurun_out/ix_tests_all.txt 2>&1 || true
grep -E "FAILED|passed|failed" gpurun_out/ix_tests_all.txt | tail -20
NNSX_X3_IRW=1 timeout -k 10 400 python -u scripts/x3_blocks_ab.py 512 3 > gpurun_out/ix_blocks_ab.txt 2>&1
cat gpurun_out/ix_blocks_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > gpurun_out/ix_tests.txt 2>&1
tail -2 gpurun_out/ix_tests.txt
timeout -k 10 300 python bench.py --sweep "" --latency-frames 0 > gpurun_out/ix_bench.json 2>/dev/null
timeout -k 10 300 python bench.py --config ssd --batch 64 --sweep "" --latency-frames 0 > gpurun_out/ix_ssd.json 2>/dev/null
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ix_bench.json gpurun_out/ix_ssd.json
