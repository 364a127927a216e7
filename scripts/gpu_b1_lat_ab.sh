#!/bin/bash
# Batch-1 live-camera latency A/B (500 fps, 600 frames per run), settings
# interleaved so box drift hits each equally.  A setting is
# "<NNSX_F32_IRW_INLAUNCH>:<NNSX_F32_SMALLM>".
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for C in ${SETTINGS:-0:0 2:1 0:1 2:0 0:0 2:1 0:1 2:0}; do
  inl=${C%%:*}; sm=${C##*:}; i=$((i + 1))
  tag=r${i}_inl${inl}_sm${sm}
  NNSX_F32_IRW_INLAUNCH=$inl NNSX_F32_SMALLM=$sm timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/b1lat_$tag.json 2> gpurun_out/b1lat_$tag.err || { echo "latency $tag failed"; tail -20 gpurun_out/b1lat_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b1lat_$tag.json')); l=d['latency_us']; print('$tag p50 %.1f p99 %.1f device %.1f' % (l['p50'], l['p99'], d['filter_device_us_median']))"
done
