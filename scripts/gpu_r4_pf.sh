#!/bin/bash
# GEMM register-prefetch A/B: numerics (both variants), micro-bench, PoseNet / MobileNetV2 pipelines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q -k "pw_conv" --timeout 120 --timeout-method thread > gpurun_out/pt_pf1.log 2>&1 && tail -1 gpurun_out/pt_pf1.log && \
NNSX_F32_GEMM_PF=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q -k "pw_conv or fused_fp32" --timeout 120 --timeout-method thread > gpurun_out/pt_pf2.log 2>&1 && tail -1 gpurun_out/pt_pf2.log || { echo "pytest failed"; tail -30 gpurun_out/pt_pf*.log; exit 1; }
timeout -k 10 150 python scripts/bench_gemm_f32.py > gpurun_out/gemm_pf1.txt 2>&1 && NNSX_F32_GEMM_PF=2 timeout -k 10 150 python scripts/bench_gemm_f32.py > gpurun_out/gemm_pf2.txt 2>&1 || exit 1
paste <(cut -c1-60 gpurun_out/gemm_pf1.txt | grep M=) <(cut -c25-60 gpurun_out/gemm_pf2.txt | grep nnsx)
for spec in "posenet:64:1" "posenet:64:2" "mbv2:512:1" "mbv2:512:2"; do
  IFS=: read c B pf <<< "$spec"
  NNSX_F32_GEMM_PF=$pf timeout -k 10 170 python bench.py --config $c --batch $B --steps 30 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/pf_${c}_$pf.log 2>&1 || { echo "bench $spec failed"; tail -20 gpurun_out/pf_${c}_$pf.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/pf_${c}_$pf.log') if l.startswith('{')][-1]); print('$c pf=$pf', d['value'], d['ms_per_step'])"
done
