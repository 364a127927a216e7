#!/bin/bash
# A/B of irw tile configurations (NNSX_IRW_SKIP hides the default entries of
# kIrwCfgs so find_irw takes the later candidates), per-layer at batch 512.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
B=${B:-512}
for SKIP in "" ${VARIANTS:-"0,1,2,3,4"}; do
  tag=${SKIP:-default}
  NNSX_IRW_SKIP=$SKIP timeout -k 10 300 python scripts/bench_ir_f32.py $B > gpurun_out/irw_ab_${tag//,/_}.txt 2>&1 || { echo "bench $tag failed"; tail -20 gpurun_out/irw_ab_${tag//,/_}.txt; exit 1; }
  echo "== skip=$tag"; grep -E "fused H=|TOTAL" gpurun_out/irw_ab_${tag//,/_}.txt
done
