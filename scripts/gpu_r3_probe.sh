#!/bin/bash
# Round-3 probes: VALU rate, H2D upload bandwidth, and a kernel + memory-copy
# trace of the default bench (where the per-step GPU idle goes).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/micro/fma_rate > gpurun_out/fma_rate.txt 2>&1 || { echo "fma_rate failed"; exit 1; }
cat gpurun_out/fma_rate.txt
timeout -k 10 180 ./scripts/micro/h2d_bw > gpurun_out/h2d_bw.txt 2>&1 || { echo "h2d_bw failed"; cat gpurun_out/h2d_bw.txt; exit 1; }
cat gpurun_out/h2d_bw.txt
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/trace_bench -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --latency-frames 0 --precision fp32 > $R/gpurun_out/trace_bench.log 2>&1 || { echo "trace failed"; tail -30 $R/gpurun_out/trace_bench.log; exit 1; }
tail -1 $R/gpurun_out/trace_bench.log | cut -c1-300
find $R/gpurun_out/trace_bench -name "*.csv" | head
