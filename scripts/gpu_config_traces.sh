#!/bin/bash
# fp32 records + one rocprofv3 kernel trace per single-GPU BASELINE config
# (bench.py --config ...), each step under its own time limit.  Summaries:
# gpurun_out/cfgtrace_<config>.txt (scripts/config_trace_report.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for spec in ${SPECS:-ssd:64 deeplab:8 posenet:64}; do
  c=${spec%%:*}; B=${spec##*:}
  cd $R && timeout -k 10 300 python3 bench.py --config $c --batch $B --steps 20 --warmup 5 --sweep "" > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log | cut -c1-300
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cfg_$c -o k --output-format csv -- python3 $R/bench.py --config $c --batch $B --steps 6 --warmup 3 --sweep "" --latency-frames 0 > $R/gpurun_out/cfgprof_$c.log 2>&1 || { echo "trace $c failed"; tail -20 $R/gpurun_out/cfgprof_$c.log; exit 1; }
  cd $R && python3 scripts/config_trace_report.py gpurun_out/cfg_$c > gpurun_out/cfgtrace_$c.txt && head -40 gpurun_out/cfgtrace_$c.txt
done
