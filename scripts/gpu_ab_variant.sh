#!/bin/bash
# same-box A/B: HEAD tree vs variants/$V (a copy of the package from another commit)
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V=${V:-base}
for rep in 1 2; do
  for spec in ${SPECS:-mbv2:512 posenet:64 deeplab:8}; do
    c=${spec%%:*}; B=${spec##*:}
    for arm in new $V; do
      if [ $arm = new ]; then b=bench.py; else b=variants/$V/bench.py; fi
      timeout -k 10 300 python $b --config $c --batch $B --sweep "" --latency-frames 0 > gpurun_out/ab_${arm}_$c.json 2>/dev/null
      echo "$rep $arm $c $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${arm}_$c.json)"
    done
  done
done
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > gpurun_out/ab_layers_new.txt 2>&1
timeout -k 10 300 python -u variants/$V/scripts/bench_ir_f32.py 512 > gpurun_out/ab_layers_$V.txt 2>&1
