#!/bin/bash
# rocprofv3 kernel-trace stats of one bench config (plus the plain-torch comparison runs).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-mbv2}; B=${B:-256}
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$CFG -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config $CFG --batch $B --steps 20 --warmup 5 ${BENCH_ARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof_$CFG.log 2>&1 || { echo "prof failed"; tail -30 $GRAFT_REPO_ROOT/gpurun_out/prof_$CFG.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_$CFG -name "*kernel_stats*"
