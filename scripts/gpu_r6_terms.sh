#!/bin/bash
# irps / irp7 numerics A/B: NNSX_IRPS_TERMS (bit 0 eight-product project, bit 1 eight-product expand,
# bit 2 compensated project accumulation) -- error vs an fp64 oracle over seeds and input distributions
# -- and block times at batch 512.
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6terms}
TERMS=${TERMS:-0 4}
mkdir -p $O
for t in $TERMS; do
  for d in relu6 normal; do
    NNSX_IRPS_TERMS=$t timeout -k 10 300 python -u scripts/x3_error_table.py --only 14,96,576,160,2 --batch 128 --seeds 6 --dist $d > $O/err_t${t}_$d.txt 2>&1
    echo "irps terms $t $d: $(tail -1 $O/err_t${t}_$d.txt)"
  done
done
for d in relu6 normal; do
  timeout -k 10 300 python -u scripts/x3_error_table.py --only 7,160,960,160,1 --batch 128 --seeds 6 --dist $d > $O/err_irp7_$d.txt 2>&1
  echo "irp7 $d: $(tail -1 $O/err_irp7_$d.txt)"
done
bash scripts/gpu_r6_layers.sh $O/layers.txt "14,96,576,160,2" $(for t in $TERMS; do echo "NNSX_IRPS_TERMS=$t"; done)
bash scripts/gpu_r6_layers.sh $O/layers.txt "7,160,960,160,1" "NNSX_IRP7=0" "NNSX_IRP7=1"
