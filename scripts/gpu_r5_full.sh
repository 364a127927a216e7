#!/bin/bash
# full GPU suite + x3 tile sweep + bench
cd "$(dirname "$0")/.."
set -e
timeout -k 10 300 python -u scripts/x3_tiles.py > gpurun_out/x3_tiles.txt 2>&1
timeout -k 10 300 python -u scripts/fan_ingest.py 8 8 32 > gpurun_out/fan_ingest.txt 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > gpurun_out/gpu_suite.txt 2>&1
tail -5 gpurun_out/gpu_suite.txt
timeout -k 10 300 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
tail -1 gpurun_out/bench_full.json | cut -c1-400
