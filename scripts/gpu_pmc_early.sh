#!/bin/bash
# PMC passes on the early fused fp32 blocks at batch 512 (scripts/pmc_f32.sh per block)
set -o pipefail
export TMPDIR=/tmp
for S in "112,16,96,24,2" "56,24,144,24,1"; do
  tag=${S//,/_}
  OUT=gpurun_out/pmc_early_$tag SHAPE=$S B=512 bash scripts/pmc_f32.sh > gpurun_out/pmc_early_$tag.txt 2>&1 || { echo "pmc $S failed"; tail -5 gpurun_out/pmc_early_$tag.txt; exit 1; }
  cat gpurun_out/pmc_early_$tag.txt
done
