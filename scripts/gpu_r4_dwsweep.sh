#!/bin/bash
# depthwise lane shapes (rows x columns per lane), stride 1 / stride 2: scripts/dw_roofline.py per pair
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dw_sweep.txt
: > $out
for pair in 0:0 42:22 44:12 81:14 82:42 22:0 24:0; do
  a=${pair%%:*}; b=${pair##*:}
  echo "# NNSX_F32_DW_S1=$a NNSX_F32_DW_S2=$b" >> $out
  NNSX_F32_DW_S1=$a NNSX_F32_DW_S2=$b timeout -k 10 120 python scripts/dw_roofline.py 2>/dev/null | grep "^B=" >> $out || { echo "run $pair failed"; exit 1; }
done
