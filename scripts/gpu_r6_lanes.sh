#!/bin/bash
# DeepLab b8 with its absorbed segmentation stage on 1 / 2 / 3 replay lanes (the stage writes only its output
# frames: DecodeStage::lane_safe), byte-exact check of the lanes against the decoder's own kernels first.
#   scripts/gpu_r6_lanes.sh [outdir]
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6lanes}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode_stage.py -q --timeout 200 --timeout-method thread > $O/decode_stage.txt 2>&1
tail -1 $O/decode_stage.txt
for rep in 1 2; do
  for l in 1 2 3; do
    NNSX_TORCH_LANES=$l timeout -k 10 300 python bench.py --config deeplab --batch 8 --steps 200 --warmup 30 --sweep "" \
      > $O/deeplab_b8_l${l}_$rep.json 2> $O/deeplab_b8_l${l}_$rep.err
    echo "lanes $l rep $rep $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/deeplab_b8_l${l}_$rep.json | tr '\n' ' ')"
  done
done
