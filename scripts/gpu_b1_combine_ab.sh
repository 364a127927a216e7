#!/bin/bash
# Batch-1 launch-count A/B: hidden-part combine (NNSX_F32_IRW_INLAUNCH 0 =
# irw_reduce launches, 2 = in-launch spread combine) x small-M GEMMs
# (NNSX_F32_SMALLM 0 = split-K GEMM + reduce launch, 1 = one-launch pw_small_f32
# and the fused head + pool).  Numerics first (bitwise / fp64 gates), then
# back-to-back graph replays and the live-camera latency probe per setting.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NNSX_F32_IRW_INLAUNCH=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "inlaunch_combine or small_m or conv_pool or top1_matches or split_k" > gpurun_out/b1c_numerics.log 2>&1 || { echo "numerics failed"; tail -30 gpurun_out/b1c_numerics.log; exit 1; }
tail -1 gpurun_out/b1c_numerics.log
for C in ${COMBOS:-"0 0" "0 1" "2 1" "0 0" "0 1" "2 1"}; do
  set -- $C
  tag=inl$1_sm$2
  NNSX_F32_IRW_INLAUNCH=$1 NNSX_F32_SMALLM=$2 timeout -k 10 200 python3 scripts/b1_graph_probe.py > gpurun_out/b1c_probe_$tag.log 2>&1 || { echo "probe $tag failed"; tail -20 gpurun_out/b1c_probe_$tag.log; exit 1; }
  echo "$tag: $(grep -E 'back-to-back' gpurun_out/b1c_probe_$tag.log)"
done
for C in ${LAT_COMBOS:-"0 0" "2 1"}; do
  set -- $C
  tag=inl$1_sm$2
  NNSX_F32_IRW_INLAUNCH=$1 NNSX_F32_SMALLM=$2 timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/b1c_lat_$tag.json 2> gpurun_out/b1c_lat_$tag.err || { echo "latency $tag failed"; tail -20 gpurun_out/b1c_lat_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b1c_lat_$tag.json')); print('$tag b1 latency', d['latency_us'], 'device', d['filter_device_us_median'])"
done
