#!/bin/bash
# Batch-1 forward time against the hidden-part count of the fp32 fused blocks
# (NNSX_F32_IRW_PARTS forces it for every block that splits; unset = irw_parts()).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in "" ${PARTS_LIST:-1 2 3 4 6}; do
  NNSX_F32_IRW_PARTS=$P timeout -k 10 200 python3 scripts/b1_graph_probe.py > gpurun_out/b1_parts_${P:-auto}.log 2>&1 || { echo "probe parts=$P failed"; tail -20 gpurun_out/b1_parts_${P:-auto}.log; exit 1; }
  echo "parts=${P:-auto}: $(grep -E 'back-to-back' gpurun_out/b1_parts_${P:-auto}.log)"
done
