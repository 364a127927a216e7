#!/bin/bash
# Round 5 evidence at HEAD defaults: configs 3-5 at the target batches and at 512, a kernel trace of
# the default bench, the per-layer split at 512, and a copy trace of the config-4 ingest.
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
for spec in ${SPECS:-ssd:64 posenet:64 deeplab:8 ssd:512 posenet:512 deeplab:512}; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --batch $B --steps 100 --warmup 20 --sweep "" > gpurun_out/cfg_${c}_b$B.log 2>&1
  tail -1 gpurun_out/cfg_${c}_b$B.log | cut -c1-240
done
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > gpurun_out/layers_b512.txt 2>&1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_head -o run --output-format csv -- \
   python3 $R/bench.py --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/gpurun_out/prof_head.log 2>&1)
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/prof_ingest -o run --output-format csv -- \
   python3 $R/scripts/fan_ingest.py 8 32 > $R/gpurun_out/prof_ingest.log 2>&1)
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u scripts/fan_ingest.py 8 8 32 > gpurun_out/fan_ingest_blit.txt 2>&1
for c in 1 2 4; do timeout -k 10 300 python -u scripts/fan_ingest.py $c 32 >> gpurun_out/fan_ingest_cams.txt 2>&1; done
echo done
