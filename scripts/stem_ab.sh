#!/bin/bash
# A/B of the fused stem + block-1 kernel variants (NNSX_STEM_WAVE) at batch 512.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in ${VARIANTS:-2 1}; do
  NNSX_STEM_WAVE=$V NNSX_IR_ONLY=stem timeout -k 10 120 python scripts/bench_ir_f32.py ${B:-512} > gpurun_out/stem_ab_$V.txt 2>&1 || { echo "stem variant $V failed"; tail -5 gpurun_out/stem_ab_$V.txt; exit 1; }
  echo "variant $V: $(grep stem gpurun_out/stem_ab_$V.txt)"
done
