#!/bin/bash
# Decoder-argmax absorption: GPU tests, the default bench and the batch-1 latency probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mbv2_f32.py tests/test_gpu_pipelines.py tests/test_gpu_elements.py > gpurun_out/t_argmax.txt 2>&1 || { tail -30 gpurun_out/t_argmax.txt; exit 1; }
tail -2 gpurun_out/t_argmax.txt
timeout -k 10 300 python bench.py > gpurun_out/bench_argmax.json 2> gpurun_out/bench_argmax.err || { tail -20 gpurun_out/bench_argmax.err; exit 1; }
cut -c1-330 gpurun_out/bench_argmax.json
timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/b1_latency_argmax.json 2> gpurun_out/b1_latency_argmax.err || { tail -20 gpurun_out/b1_latency_argmax.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b1_latency_argmax.json')); print('b1 latency', d['latency_us'], 'device', d['filter_device_us_median'])"
