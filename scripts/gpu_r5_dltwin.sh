#!/bin/bash
# DeepLab b8 with every fused block on its x3 twin (NNSX_X3_IRW=1) / expand-x3 twin (=2) vs the defaults
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
for rep in 1 2; do
  for m in 0 1 2; do
    if [ $m = 0 ]; then unset NNSX_X3_IRW; else export NNSX_X3_IRW=$m; fi
    timeout -k 10 300 python bench.py --config deeplab --batch 8 --sweep "" --latency-frames 0 > gpurun_out/dltwin.json 2>/dev/null
    echo "$rep x3irw=$m deeplab b8 $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/dltwin.json)"
  done
done
for m in 1 2; do
  (cd /tmp && NNSX_X3_IRW=$m timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ct_dltwin$m -o run --output-format csv -- \
     python3 $R/bench.py --config deeplab --batch 8 --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/gpurun_out/ct_dltwin$m.log 2>&1)
done
