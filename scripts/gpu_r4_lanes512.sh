#!/bin/bash
# Replay lanes at the headline batch (and 128): bench.py frames/s with NNSX_TORCH_LANES=1/2/3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/lanes512.txt
: > $out
for B in ${BATCHES:-512 128}; do
  for L in ${LANES:-1 3 2}; do
    NNSX_TORCH_LANES=$L timeout -k 10 200 python bench.py --batch $B --steps ${STEPS:-100} --warmup 10 --sweep "" --latency-frames 0 ${QARGS} > gpurun_out/lanes_b${B}_l$L.log 2>&1 || { echo "bench B=$B L=$L failed"; tail -20 gpurun_out/lanes_b${B}_l$L.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/lanes_b${B}_l$L.log') if l.startswith('{')][-1]); print('b$B lanes=$L', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'), d.get('p50_latency_ms'))" | tee -a $out
  done
done
