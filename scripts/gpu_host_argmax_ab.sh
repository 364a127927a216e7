#!/bin/bash
# Absorbed-argmax indices copied to pinned host memory after each replay
# (NNSX_TORCH_HOST_ARGMAX=1) vs a device clone read back by the decoder (0): GPU tests,
# then the batch-1 live latency, settings interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NNSX_TORCH_HOST_ARGMAX=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for H in ${HOSTS:-0 1 0 1 0 1}; do
  NNSX_TORCH_HOST_ARGMAX=$H timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/hargmax_lat_$H.json 2> gpurun_out/hargmax_lat_$H.err || { echo "latency host_argmax=$H failed"; tail -20 gpurun_out/hargmax_lat_$H.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/hargmax_lat_$H.json')); l=d['latency_us']; print('host_argmax=$H p50 %.1f p99 %.1f device %.1f' % (l['p50'], l['p99'], d['filter_device_us_median']))"
done
