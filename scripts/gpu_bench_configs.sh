#!/bin/bash
# Bench every single-GPU BASELINE config; each step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in ${SPECS:-mbv2:256 ssd:64 deeplab:8 posenet:64}; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --batch $B --steps ${STEPS:-20} --warmup ${WARMUP:-5} > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -30 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log | cut -c1-400
done
