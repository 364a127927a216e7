#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in ${BATCHES:-1 16 64}; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 --batch $B ${BENCH_ARGS} > gpurun_out/bench_b$B.log 2>&1 || { echo "bench B=$B failed"; tail -30 gpurun_out/bench_b$B.log; exit 1; }
  tail -1 gpurun_out/bench_b$B.log
done
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --batch ${PROF_BATCH:-64} ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof.log; exit 1; }
  find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head
fi
