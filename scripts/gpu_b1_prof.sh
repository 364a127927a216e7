#!/bin/bash
# Batch-1 forward under rocprofv3 (kernel trace + stats): back-to-back graph
# replays of the fp32 engine (scripts/b1_graph_probe.py), and the live-camera
# latency probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/b1prof -o b1 --output-format csv -- python3 $R/scripts/b1_graph_probe.py > $R/gpurun_out/b1prof.log 2>&1 || { echo "b1 prof failed"; tail -20 $R/gpurun_out/b1prof.log; exit 1; }
grep -E "graph replay|eager" $R/gpurun_out/b1prof.log
cd $R && timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/b1_latency.json 2> gpurun_out/b1_latency.err || { echo "b1 latency failed"; tail -20 gpurun_out/b1_latency.json; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b1_latency.json')); print('b1 latency', d['latency_us'], 'device', d['filter_device_us_median'])"
