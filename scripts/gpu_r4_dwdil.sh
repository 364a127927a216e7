#!/bin/bash
# dilation-2 depthwise as 4x4 column lanes: gates, kernel A/B, DeepLab benches A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dw or deeplab" > gpurun_out/dwdil_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/dwdil_pytest.log; exit 1; }
tail -1 gpurun_out/dwdil_pytest.log
timeout -k 10 120 python scripts/dw_roofline.py 2>/dev/null | grep "^B=" > gpurun_out/dwdil_roof.txt
NNSX_F32_DW_DIL_COL=0 timeout -k 10 120 python scripts/dw_roofline.py 2>/dev/null | grep "^B=" > gpurun_out/dwdil_roof_off.txt
out=gpurun_out/dwdil_bench.txt
: > $out
for B in 8 32; do
  for v in 1 0; do
    NNSX_F32_DW_DIL_COL=$v timeout -k 10 200 python bench.py --config deeplab --batch $B --steps 40 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/dwdil_b${B}_$v.log 2>&1 || { echo "bench $B $v failed"; tail -20 gpurun_out/dwdil_b${B}_$v.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dwdil_b${B}_$v.log') if l.startswith('{')][-1]); print('deeplab b$B dil_col=$v', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))" | tee -a $out
  done
done
