#!/bin/bash
# Pipelined-expand (VAR = 1) irw variants: numerics under the variant selection,
# then per-layer A/B at batch 512 against the defaults.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_ALL=${SKIP_ALL:-0,1,2,3,13,14,15,16}
NNSX_IRW_SKIP=$SKIP_ALL timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "ir_block_f32 or bench_batch_matches" > gpurun_out/pipe_numerics.log 2>&1 || { echo "numerics failed"; tail -30 gpurun_out/pipe_numerics.log; exit 1; }
tail -2 gpurun_out/pipe_numerics.log
NNSX_STEM_WAVE=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "stem_ir1 or bench_batch_matches" > gpurun_out/spipe_numerics.log 2>&1 || { echo "stem numerics failed"; tail -30 gpurun_out/spipe_numerics.log; exit 1; }
tail -2 gpurun_out/spipe_numerics.log
NNSX_STEM_WAVE=3 timeout -k 10 300 python scripts/bench_ir_f32.py 512 > gpurun_out/spipe_ab.txt 2>&1 || { echo "stem bench failed"; tail -20 gpurun_out/spipe_ab.txt; exit 1; }
echo "== stem pipelined"; grep -E "stem|TOTAL" gpurun_out/spipe_ab.txt
VARIANTS=${VARIANTS:-"0,1,13,14,15,16 $SKIP_ALL"} bash scripts/irw_ab.sh
