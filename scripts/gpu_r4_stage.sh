#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_stage.py tests/test_gpu_mbv2_f32.py tests/test_gpu_comm.py tests/test_gpu_models_f32.py tests/test_gpu_elements.py tests/test_gpu_decoders_golden.py tests/test_gpu_pipelines.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_stage.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_stage.log; exit 1; }
tail -3 gpurun_out/pytest_stage.log
# A/B of the new fusions (env toggles) on the config benches
for spec in "posenet:64:NNSX_POSENET_DWPW=0" "deeplab:8:NNSX_DWPW_DILATED=0" "ssd:64:NNSX_SSD_SEP_HEADS=0"; do
  IFS=: read c B envv <<< "$spec"
  env $envv timeout -k 10 300 python bench.py --config $c --batch $B --steps 20 --warmup 5 --sweep "" --latency-frames 0 > gpurun_out/bench_${c}_b${B}_off.log 2>&1 || { echo "bench $c off failed"; tail -20 gpurun_out/bench_${c}_b${B}_off.log; exit 1; }
  echo "$envv: $(tail -1 gpurun_out/bench_${c}_b${B}_off.log | cut -c1-200)"
done
bash scripts/gpu_r4_configs.sh
