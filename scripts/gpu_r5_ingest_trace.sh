#!/bin/bash
# host-side timeline of the config-4 ingest at batch 8 (HIP API + copies + kernels)
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
for c in 1 8; do
(cd /tmp && timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace -d $R/gpurun_out/tr_ingest$c -o run --output-format csv -- \
   python3 $R/scripts/fan_ingest.py $c 8 > $R/gpurun_out/tr_ingest$c.log 2>&1)
done
tail -1 gpurun_out/tr_ingest1.log; tail -1 gpurun_out/tr_ingest8.log
