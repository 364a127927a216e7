#!/bin/bash
# replay lanes re-measured (no in-launch combine while lanes share the device)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q -k "lanes or decoder_argmax or benched" --timeout 120 --timeout-method thread > gpurun_out/pt_lanes2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pt_lanes2.log; exit 1; }
tail -1 gpurun_out/pt_lanes2.log
for B in 8 16 32; do for L in 1 3; do
  NNSX_TORCH_LANES=$L timeout -k 10 170 python3 bench.py --batch $B --steps 400 --warmup 20 --latency-frames 0 --sweep "" > gpurun_out/lanes2_b${B}_l$L.log 2>&1 || { echo "bench b$B lanes $L failed"; tail -20 gpurun_out/lanes2_b${B}_l$L.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/lanes2_b${B}_l$L.log') if l.startswith('{')][-1]); print('b$B lanes=$L', d['value'], d['ms_per_step'], d['gpu_invoke_ms_median'], d['p50_latency_ms'])"
done; done
