#!/bin/bash
# kernel traces of configs 3-5 at their target batches (HEAD defaults)
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
for spec in ${SPECS:-ssd:64 posenet:64 deeplab:8 deeplab:1}; do
  c=${spec%%:*}; B=${spec##*:}
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ct_${c}_b$B -o run --output-format csv -- \
     python3 $R/bench.py --config $c --batch $B --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/gpurun_out/ct_${c}_b$B.log 2>&1)
  tail -1 gpurun_out/ct_${c}_b$B.log | cut -c1-200
done
