#!/bin/bash
# irw_f32 stride-2 tiles with per-quad hidden planes one cell apart (GSH): fp32 block numerics, per-block times at
# batch 512, LDS counters of the 56 -> 28 and 112 -> 56 blocks, the headline bench.
#   scripts/gpu_r6_irw2.sh [outdir]
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6irw2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_x3.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
tail -1 $O/tests.txt
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > $O/layers_b512.txt 2>&1
grep -E "H=112|H=56|TOTAL" $O/layers_b512.txt
for spec in "56,24,144,32,2 irw_f32" "112,16,96,24,2 irw_f32"; do
  set -- $spec
  tag=$(echo "$1_$2" | tr ',' '_')
  OUT=$O/$tag SHAPE=$1 B=512 KERNEL=$2 bash scripts/pmc_f32.sh > $O/$tag.txt 2>&1
  echo "== $1 $2"; tail -2 $O/$tag.txt
done
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-300; echo
