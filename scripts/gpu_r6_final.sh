#!/bin/bash
# Round-6 records in one call: GPU suite, default bench (100 + 20), the other configs at their target batches,
# windowed headline kernel stats, per-layer split (x3 defaults and native fp32), x3 error table, lowered-engine bench.
#   scripts/gpu_r6_final.sh [outdir]
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6final}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
rc=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_suite.txt 2>&1 || rc=$?
tail -2 $O/gpu_suite.txt
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-300; echo
for c in "ssd 64" "deeplab 8" "posenet 64" "deeplab_fan 8" "posenet_multi 64"; do
  set -- $c
  timeout -k 10 300 python bench.py --config $1 --batch $2 --steps 100 --warmup 20 --sweep "" > $O/cfg_$1_b$2.json 2> $O/cfg_$1_b$2.err
  echo "$1 b$2 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/cfg_$1_b$2.json | tr '\n' ' ')"
done
timeout -k 10 400 python bench.py --engine lowered --sweep "" --latency-frames 0 > $O/bench_lowered.json 2> $O/bench_lowered.err
echo "lowered $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"lowered": "[^"]*"' $O/bench_lowered.json | tr '\n' ' ')"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $R/$O/prof -o run --output-format csv -- \
   python3 $R/bench.py --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/$O/prof.log 2>&1)
python3 scripts/kstats.py $O/prof --window --per-step 20 > $O/kstats_window.txt
head -4 $O/kstats_window.txt
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > $O/layers_b512.txt 2>&1
NNSX_F32_MATH=fp32 timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > $O/layers_b512_native.txt 2>&1
timeout -k 10 300 python -u scripts/x3_error_table.py --batch 512 > $O/x3_error_table.txt 2>&1
tail -1 $O/x3_error_table.txt
