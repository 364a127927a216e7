#!/bin/bash
# x3 defaults: tests, model A/B, bench
cd "$(dirname "$0")/.."
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_mbv2_f32.py -q --timeout 120 --timeout-method thread > gpurun_out/x3_tests3.txt 2>&1
tail -3 gpurun_out/x3_tests3.txt
timeout -k 10 300 python -u scripts/x3_ab.py --rounds 3 > gpurun_out/x3_model3.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_x3.json 2> gpurun_out/bench_x3.err || exit 1
tail -1 gpurun_out/bench_x3.json
