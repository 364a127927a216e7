#!/bin/bash
# One GPU-box session: tests, bench, profile.  Every GPU step has its own time limit.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEP=${1:-all}
if [ "$STEP" = "all" ] || [ "$STEP" = "test" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -50 gpurun_out/pytest_gpu.log; exit 1; }
  tail -5 gpurun_out/pytest_gpu.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "bench" ]; then
  timeout -k 10 600 python bench.py --steps 30 --warmup 10 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -50 gpurun_out/bench.log; exit 1; }
  tail -3 gpurun_out/bench.log
fi
