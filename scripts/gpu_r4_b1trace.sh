#!/bin/bash
# kernel traces of the batch-1 live-camera runs of DeepLab and PoseNet
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for spec in deeplab:100 posenet:250; do
  c=${spec%%:*}; f=${spec##*:}
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/b1tr_$c -o tr -- python3 $R/bench.py --config $c --batch 8 --steps 2 --warmup 1 --sweep "" --latency-fps $f --latency-frames 60 > $R/gpurun_out/b1tr_$c.log 2>&1) || { echo "trace $c failed"; tail -20 $R/gpurun_out/b1tr_$c.log; exit 1; }
done
echo done
