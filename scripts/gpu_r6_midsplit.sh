#!/bin/bash
# Split-K for mid-size GEMM grids (NNSX_GEMM_MIDSPLIT=1: 128-511 tiles in two k-slices, residual added by the reduce):
# fp32 numerics under the switch, then each config with it off / on (DeepLab b8's 8712 x 960 -> 160 projects).
#   scripts/gpu_r6_midsplit.sh [outdir]
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6mid}
mkdir -p $O
export TMPDIR=/tmp
NNSX_GEMM_MIDSPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_x3.py tests/test_gpu_models_f32.py tests/test_gpu_decode_stage.py -q -x --timeout 300 --timeout-method thread > $O/tests_mid.txt 2>&1
tail -1 $O/tests_mid.txt
for rep in 1 2; do
  for c in "deeplab 8" "ssd 64" "posenet 64"; do
    set -- $c
    for m in 0 1; do
      NNSX_GEMM_MIDSPLIT=$m timeout -k 10 300 python bench.py --config $1 --batch $2 --steps 200 --warmup 30 --sweep "" > $O/${1}_m${m}_r${rep}.json 2> $O/${1}_m${m}_r${rep}.err
      echo "$1 b$2 mid=$m rep $rep $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/${1}_m${m}_r${rep}.json | tr '\n' ' ')"
    done
  done
done
