#!/bin/bash
# PMC of one fused block, native fp32 kernel vs the x3 kernel (batch 512)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
S=${S:-14,64,384,64,1}
n=$(echo $S | tr ',' '_')
for X in 0 1; do
  OUT=gpurun_out/pmc_x3_${n}_$X NNSX_X3_IRW=$X SHAPE=$S B=512 KERNEL=irw_ bash scripts/pmc_f32.sh > gpurun_out/pmc_x3_${n}_$X.txt 2>&1 || { echo "pmc $X failed"; tail -5 gpurun_out/pmc_x3_${n}_$X.txt; exit 1; }
  cat gpurun_out/pmc_x3_${n}_$X.txt
done
