#!/bin/bash
# per-layer A/B at batch 512: scripts/gpu_r6_layers.sh <out file> "<shapes>" "<variant>" ["<variant>" ...]
# shapes: space-separated H,cin,hid,cout,stride; a variant: space-separated NNSX_* settings (or NONE=1)
set -eo pipefail
cd "$(dirname "$0")/.."
out=$1; shapes=$2; shift 2
mkdir -p "$(dirname "$out")"
for f in $shapes; do
  for v in "$@"; do
    r=$(env $v NNSX_IR_ONLY=$f timeout -k 10 120 python -u scripts/bench_ir_f32.py 512 2>&1 | grep fused)
    echo "$v | $r" | tee -a "$out"
  done
done
