#!/bin/bash
# Round 4, third config pass: every single-GPU config at the current defaults (incl. the
# batch-1 live-camera latency), DeepLab lanes A/B, GEMM tile A/B on PoseNet / SSD, upload bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
one() {  # name, config, batch, extra env...
  local name=$1 c=$2 B=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --config $c --batch $B --steps 30 --warmup 10 --sweep "" > gpurun_out/cfg3_$name.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/cfg3_$name.log; return 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/cfg3_$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'), d.get('p50_latency_ms'), d.get('p50_latency_ms_b1'), d.get('p99_latency_ms_b1'))"
}
one ssd64 ssd 64 NNSX_NONE=1 && one deeplab8 deeplab 8 NNSX_NONE=1 && one deeplab16 deeplab 16 NNSX_NONE=1 && \
one deeplab32 deeplab 32 NNSX_NONE=1 && one posenet64 posenet 64 NNSX_NONE=1 && \
one deeplab8_l1 deeplab 8 NNSX_TORCH_LANES=1 && one posenet64_g128128 posenet 64 NNSX_F32_GEMM_TILE=128128 && \
one posenet64_g64128 posenet 64 NNSX_F32_GEMM_TILE=64128 && one ssd64_g128128 ssd 64 NNSX_F32_GEMM_TILE=128128 && \
one posenet32 posenet 32 NNSX_NONE=1 && one ssd32 ssd 32 NNSX_NONE=1 || exit 1
for w in 513:8 257:64; do
  timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 2>&1 | grep width || exit 1
done
