#!/bin/bash
# One GPU-box session.  Each GPU step has its own time limit; the first failing
# step ends the session (no retries).  STEPS: comma list of
#   f32      new fp32 kernel tests            (tests/test_gpu_mbv2_f32.py)
#   test     the whole GPU suite
#   smoke    __graft_entry__.smoke()
#   bench    bench.py (BENCH_ARGS)
#   prof     rocprofv3 kernel stats of bench.py (PROF_ARGS)
#   irf32    per-layer fp32 engine micro-benchmark (scripts/bench_ir_f32.py)
#   latprof  rocprofv3 host+device trace of the batch-1 latency run
#   irvar    bench_ir_f32 once per IR_VARIANTS env set
#   pmcf32   PMC counter passes over it (scripts/pmc_f32.sh; SHAPE=, KERNEL=)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-f32,test,smoke,bench}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
for s in ${STEPS//,/ }; do
  case $s in
    f32)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_f32.log 2>&1 || { echo "f32 tests failed"; tail -60 gpurun_out/pytest_f32.log; exit 1; }
      tail -3 gpurun_out/pytest_f32.log ;;
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
      tail -3 gpurun_out/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
      tail -2 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
      tail -1 gpurun_out/bench.log ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py ${PROF_ARGS} > $R/gpurun_out/prof.log 2>&1) || { echo "prof failed"; tail -30 gpurun_out/prof.log; exit 1; }
      find gpurun_out/prof -name "*kernel_stats.csv" ;;
    latprof)
      # host (HIP API) + device timeline of the batch-1 latency run
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $R/gpurun_out/latprof -o run --output-format csv -- python3 $R/bench.py --precision fp32 --steps 3 --warmup 2 --latency-frames 200 > $R/gpurun_out/latprof.log 2>&1) || { echo "latprof failed"; tail -30 gpurun_out/latprof.log; exit 1; }
      tail -1 gpurun_out/latprof.log | cut -c1-300 ;;
    irf32)
      timeout -k 10 300 python -u scripts/bench_ir_f32.py ${IR_B:-128} > gpurun_out/bench_ir_f32.log 2>&1 || { echo "bench_ir_f32 failed"; tail -30 gpurun_out/bench_ir_f32.log; exit 1; }
      cat gpurun_out/bench_ir_f32.log ;;
    irvar)
      # IR_VARIANTS: ';'-separated env assignments, one bench_ir_f32 run each
      IFS=';' read -ra VARS <<< "${IR_VARIANTS:-NNSX_F32_IRW=1}"
      for V in "${VARS[@]}"; do
        env $V timeout -k 10 300 python -u scripts/bench_ir_f32.py ${IR_B:-128} > gpurun_out/irvar.log 2>&1 || { echo "irvar $V failed"; tail -30 gpurun_out/irvar.log; exit 1; }
        echo "== $V"; grep -v amdgpu.ids gpurun_out/irvar.log
      done ;;
    gemmf32)
      for R in ${DW_ROWS:-4}; do
        NNSX_F32_DW_ROWS=$R timeout -k 10 300 python -u scripts/bench_gemm_f32.py ${IR_B:-128} > gpurun_out/bench_gemm_f32_r$R.log 2>&1 || { echo "bench_gemm_f32 failed"; tail -30 gpurun_out/bench_gemm_f32_r$R.log; exit 1; }
        echo "== dw rows $R"; cat gpurun_out/bench_gemm_f32_r$R.log
      done ;;
    pmcf32)
      timeout -k 10 600 bash scripts/pmc_f32.sh > gpurun_out/pmc_f32.log 2>&1 || { echo "pmc failed"; tail -30 gpurun_out/pmc_f32.log; exit 1; }
      cat gpurun_out/pmc_f32.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
