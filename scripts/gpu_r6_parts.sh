#!/bin/bash
# Hidden-channel parts of the wave-split kernels on 128-255 tiles (NNSX_IRW_PARTS_MID=2 default / 3 / 4): DeepLab b8's 33x33
# blocks (200 tiles, 400 workgroups at 2 parts).  Numerics under 4 parts first.
#   scripts/gpu_r6_parts.sh [outdir]
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6parts}
mkdir -p $O
export TMPDIR=/tmp
NNSX_IRW_PARTS_MID=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py tests/test_gpu_decode_stage.py -q -x --timeout 300 --timeout-method thread > $O/tests_p4.txt 2>&1
tail -1 $O/tests_p4.txt
for rep in 1 2; do
  for p in 2 4 3; do
    NNSX_IRW_PARTS_MID=$p timeout -k 10 300 python bench.py --config deeplab --batch 8 --steps 200 --warmup 30 --sweep "" > $O/dl_p${p}_r${rep}.json 2> $O/dl_p${p}_r${rep}.err
    echo "deeplab b8 parts=$p rep $rep $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/dl_p${p}_r${rep}.json | tr '\n' ' ')"
  done
done
