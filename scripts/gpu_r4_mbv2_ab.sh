#!/bin/bash
# Round 4: headline-engine A/B (layer timings + short bench) of the candidate changes,
# then the PMC of the line-buffer stem.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/bench_ir_f32.py 512 > gpurun_out/r4_fp32_layers_b512.txt 2>&1 || { echo "layers failed"; tail -20 gpurun_out/r4_fp32_layers_b512.txt; exit 1; }
cat gpurun_out/r4_fp32_layers_b512.txt
NNSX_IRW_SKIP=6 timeout -k 10 300 python3 scripts/bench_ir_f32.py 512 > gpurun_out/r4_fp32_layers_b512_t77.txt 2>&1 || { echo "layers t714 failed"; exit 1; }
grep -E "H=14|TOTAL" gpurun_out/r4_fp32_layers_b512_t77.txt
run() {  # name, env... (BENCH_ARGS: extra bench.py arguments)
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 --latency-frames 0 --sweep "" $BENCH_ARGS > gpurun_out/ab_$name.log 2>&1 || { echo "ab $name failed"; tail -20 gpurun_out/ab_$name.log; return 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['ms_per_step'], d['gpu_invoke_ms_median'], d['p50_latency_ms'])"
}
run base NNSX_NONE=1 && run t77_64 NNSX_IRW_SKIP=6 && run headpool_off NNSX_F32_HEAD_POOL=0 && run dwpw_all NNSX_DWPW_ALL=1 && run gemm128 NNSX_F32_GEMM_TILE=128128 && run base2 NNSX_NONE=1 && BENCH_ARGS="--queue 1 --queue-in 1" run q11 NNSX_NONE=1 && BENCH_ARGS="--queue 2 --queue-in 1" run q21 NNSX_NONE=1 || exit 1
for S in stem stemband; do
  OUT=gpurun_out/pmc_$S SHAPE=$S B=512 bash scripts/pmc_f32.sh > gpurun_out/pmc_$S.txt 2>&1 || { echo "pmc $S failed"; tail -5 gpurun_out/pmc_$S.txt; exit 1; }
  cat gpurun_out/pmc_$S.txt
done
