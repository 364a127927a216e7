#!/bin/bash
# Round 4: every BASELINE config on one GPU (incl. the multi-rank configs at N=1) plus
# kernel traces of DeepLab / PoseNet (padded-frame upload path).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in ${SPECS:-ssd:64 deeplab:8 deeplab:16 deeplab:32 posenet:64 deeplab_fan:8 posenet_multi:64}; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --batch $B --steps ${STEPS:-20} --warmup ${WARMUP:-5} --sweep "" > gpurun_out/bench_${c}_b$B.log 2>&1 || { echo "bench $c failed"; tail -30 gpurun_out/bench_${c}_b$B.log; exit 1; }
  tail -1 gpurun_out/bench_${c}_b$B.log | cut -c1-300
done
for spec in ${TRACES:-deeplab:8 posenet:64}; do
  c=${spec%%:*}; B=${spec##*:}
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$c -o $c -- \
     python $GRAFT_REPO_ROOT/bench.py --config $c --batch $B --steps 10 --warmup 3 --sweep "" --latency-frames 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$c.log 2>&1) || { echo "trace $c failed"; exit 1; }
done
echo done
