#!/bin/bash
# hipBLASLt for the plain fp32 GEMMs: numerics, then the configs and the headline A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_blaslt.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_blaslt.log; exit 1; }
tail -1 gpurun_out/pytest_blaslt.log
one() {  # name, config, batch, env...
  local name=$1 c=$2 B=$3; shift 3
  env "$@" timeout -k 10 300 python bench.py --config $c --batch $B --steps 30 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/bl_$name.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/bl_$name.log; return 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bl_$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))"
}
one posenet_on posenet 64 NNSX_NONE=1 && one posenet_off posenet 64 NNSX_F32_BLASLT=0 && one posenet_nodefer posenet 64 NNSX_DEFER_ACT=0 && \
one ssd_on ssd 64 NNSX_NONE=1 && one ssd_off ssd 64 NNSX_F32_BLASLT=0 && \
one deeplab8_on deeplab 8 NNSX_NONE=1 && one deeplab8_off deeplab 8 NNSX_F32_BLASLT=0 && \
one deeplab32_on deeplab 32 NNSX_NONE=1 && \
one mbv2_on mbv2 512 NNSX_NONE=1 && one mbv2_off mbv2 512 NNSX_F32_BLASLT=0 || exit 1
