#!/bin/bash
# Batch-1 single-frame upload: copy engine (hipMemcpyAsync, default) vs the
# gather kernel reading the pinned frame over the bus (NNSX_CONV_KERNEL_UPLOAD=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NNSX_CONV_KERNEL_UPLOAD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "decoder_argmax_absorbed or benched_launch_string" > gpurun_out/upload_numerics.log 2>&1 || { echo "numerics failed"; tail -30 gpurun_out/upload_numerics.log; exit 1; }
tail -1 gpurun_out/upload_numerics.log
for U in ${UPLOADS:-0 1 0 1 0 1}; do
  NNSX_CONV_KERNEL_UPLOAD=$U timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/upload_lat_$U.json 2> gpurun_out/upload_lat_$U.err || { echo "latency upload=$U failed"; tail -20 gpurun_out/upload_lat_$U.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/upload_lat_$U.json')); l=d['latency_us']; print('kernel_upload=$U p50 %.1f p99 %.1f device %.1f' % (l['p50'], l['p99'], d['filter_device_us_median']))"
done
