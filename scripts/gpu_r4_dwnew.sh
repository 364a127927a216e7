#!/bin/bash
# 4x4 / 2x2 depthwise lanes as the default: depthwise + model gates, then the config benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dw or sep_heads or models_f32 or posenet or ssd or deeplab or mbv2_f32" > gpurun_out/dwnew_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/dwnew_pytest.log; exit 1; }
tail -1 gpurun_out/dwnew_pytest.log
timeout -k 10 120 python scripts/dw_roofline.py 2>/dev/null | grep "^B=" > gpurun_out/dwnew_roof.txt
out=gpurun_out/dwnew_bench.txt
: > $out
for spec in mbv2:512 posenet:64 ssd:64 deeplab:8 posenet:512; do
  c=${spec%%:*}; B=${spec##*:}
  for v in 44:22 0:0; do
    a=${v%%:*}; b=${v##*:}
    NNSX_F32_DW_S1=$a NNSX_F32_DW_S2=$b timeout -k 10 200 python bench.py --config $c --batch $B --steps 60 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/dwnew_${c}_$a.log 2>&1 || { echo "bench $c $a failed"; tail -20 gpurun_out/dwnew_${c}_$a.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dwnew_${c}_$a.log') if l.startswith('{')][-1]); print('$c b$B dw=$a/$b', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))" | tee -a $out
  done
done
