#!/bin/bash
# DeepLab at small batches: replay lanes auto (3 below 33 frames / 8 MB) vs 1
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dllanes.txt
: > $out
for B in 8 16; do
  for L in 1 3 1 3; do
    NNSX_TORCH_LANES=$L timeout -k 10 200 python bench.py --config deeplab --batch $B --steps 60 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/dll_b${B}_$L.log 2>&1 || { echo "bench $B $L failed"; tail -20 gpurun_out/dll_b${B}_$L.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dll_b${B}_$L.log') if l.startswith('{')][-1]); print('deeplab b$B lanes=$L', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'), d.get('p50_latency_ms'))" | tee -a $out
  done
done
