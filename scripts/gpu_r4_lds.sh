#!/bin/bash
# Round 4: LDS-conflict-free depthwise reads (stem planes 16-quad aligned + global
# LUT; irw pixel orders / deinterleaved stride-2 hidden images): numerics,
# layer timings, the bench, and the PMC of the stem and the early blocks.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_lds.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_lds.log; exit 1; }
tail -2 gpurun_out/pytest_lds.log
timeout -k 10 300 python3 scripts/bench_ir_f32.py 512 > gpurun_out/r4_fp32_layers_b512_lds.txt 2>&1 || { echo "layers failed"; tail -20 gpurun_out/r4_fp32_layers_b512_lds.txt; exit 1; }
cat gpurun_out/r4_fp32_layers_b512_lds.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --latency-frames 0 --sweep "" > gpurun_out/bench_lds.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_lds.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bench_lds.log') if l.startswith('{')][-1]); print('bench', d['value'], d['ms_per_step'], d['gpu_invoke_ms_median'], d['p50_latency_ms'])"
for S in stem "112,16,96,24,2" "56,24,144,24,1" "56,24,144,32,2" "28,32,192,32,1"; do
  n=$(echo $S | tr ',' '_')
  OUT=gpurun_out/pmc_lds_$n SHAPE=$S B=512 bash scripts/pmc_f32.sh > gpurun_out/pmc_lds_$n.txt 2>&1 || { echo "pmc $S failed"; tail -5 gpurun_out/pmc_lds_$n.txt; exit 1; }
  cat gpurun_out/pmc_lds_$n.txt
done
