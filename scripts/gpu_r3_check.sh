#!/bin/bash
# GPU gate: gpu tests, smoke, default bench (each step under its own limit).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TESTS:-tests}
timeout -k 10 1200 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Error|error" gpurun_out/pytest_gpu.log | head -20; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
if [ -z "$NO_SMOKE" ]; then
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
fi
timeout -k 10 600 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
