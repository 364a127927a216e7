#!/bin/bash
# host-side view of the sustained headline: roctx range per element chain call (NNSX_TRACERS=roctx) with the
# kernel and memory-copy traces of a 100-step bench.py run, for finding what the GPU waits for between steps.
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6host}
mkdir -p $O
export TMPDIR=/tmp NNSX_BENCH_SERIES=1 NNSX_TRACERS=roctx
R=$PWD
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace ${EXTRA_TRACE:-} -d $R/$O/prof -o run --output-format csv -- \
   python3 $R/bench.py --sweep "" --latency-frames 0 > $R/$O/bench.json 2> $R/$O/bench.err)
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench.json | tr '\n' ' '; echo
ls $O/prof/*
