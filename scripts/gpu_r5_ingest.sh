#!/bin/bash
# config-4 ingest after the per-run padded DMA: converter tests, then the fan-in bench
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_elements.py -q -x --timeout 120 --timeout-method thread -k "converter" > gpurun_out/ingest_tests.txt 2>&1
tail -2 gpurun_out/ingest_tests.txt
timeout -k 10 300 python -u scripts/fan_ingest.py 8 8 32 > gpurun_out/fan_ingest2.txt 2>&1
timeout -k 10 300 python -u scripts/fan_ingest.py 1 8 32 >> gpurun_out/fan_ingest2.txt 2>&1
cat gpurun_out/fan_ingest2.txt
