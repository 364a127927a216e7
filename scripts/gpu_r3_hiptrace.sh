#!/bin/bash
# Host-side view of the bench step: HIP runtime API + kernel + copy trace of a
# short default bench run (where the per-step GPU idle comes from).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/hiptrace -o run --output-format csv -- python3 $R/bench.py --steps 12 --warmup 4 --latency-frames 0 --sweep "" > $R/gpurun_out/hiptrace.log 2>&1 || { echo "trace failed"; tail -30 $R/gpurun_out/hiptrace.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/hiptrace.log
ls -la $R/gpurun_out/hiptrace/*
python3 $R/scripts/stall_report.py $R/gpurun_out/hiptrace > $R/gpurun_out/stall_report.txt 2>&1 && tail -22 $R/gpurun_out/stall_report.txt
