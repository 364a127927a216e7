#!/bin/bash
# irpp (pipelined image-per-workgroup 14x14 block) A/B: accuracy gate per variant,
# per-layer times at batch 512 for every variant and phase order.
#   scripts/gpu_r6_irpp.sh [outdir]
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6irpp}
mkdir -p $O
export TMPDIR=/tmp
for v in "NNSX_IRP_PIPE=1" "NNSX_IRP_PIPE=1 NNSX_IRP_TPW=1"; do
  rc=0
  env $v timeout -k 10 300 python -u -m pytest tests/test_gpu_irp.py -q --timeout 200 --timeout-method thread -k "not wave_split" > $O/tests.txt 2>&1 || rc=$?
  echo "$v: $(tail -1 $O/tests.txt)" | tee -a $O/tests_summary.txt
  [ $rc -le 1 ] || exit $rc
done
for f in 14,64,384,64,1 14,64,384,96,1 14,96,576,96,1; do
  for v in "NNSX_IRP_PIPE=0" "NNSX_IRP_PIPE=1 NNSX_IRP_TPW=2 NNSX_IRP_ORDER=1" "NNSX_IRP_PIPE=1 NNSX_IRP_TPW=2 NNSX_IRP_ORDER=0" \
           "NNSX_IRP_PIPE=1 NNSX_IRP_TPW=2 NNSX_IRP_ORDER=2" "NNSX_IRP_PIPE=1 NNSX_IRP_TPW=1 NNSX_IRP_ORDER=1" \
           "NNSX_IRP_PIPE=1 NNSX_IRP_TPW=1 NNSX_IRP_ORDER=0"; do
    echo "$v | $(env $v NNSX_IR_ONLY=$f timeout -k 10 120 python -u scripts/bench_ir_f32.py 512 2>&1 | grep fused)" | tee -a $O/layers.txt
  done
done
