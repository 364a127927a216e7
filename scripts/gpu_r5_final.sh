#!/bin/bash
# Round-5 records at HEAD defaults: GPU suite, default bench, configs 3-5 (target batches and 512),
# kernel stats of the default bench and of each config, per-layer split at batch 512
# (PART=1: suite, bench, configs; PART=2: per-layer split and kernel traces; unset: both)
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/final
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/final
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > $O/gpu_suite.txt 2>&1
tail -2 $O/gpu_suite.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-220
for spec in ssd:64 posenet:64 deeplab:8 ssd:512 posenet:512 deeplab:512 deeplab_fan:8 posenet_multi:64; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --batch $B --steps 100 --warmup 20 --sweep "" > $O/cfg_${c}_b$B.json 2> $O/cfg_${c}_b$B.err
  echo "$c b$B $(grep -h -o '"value": [0-9.]*' $O/cfg_${c}_b$B.json) $(grep -h -o '"ms_per_step": [0-9.]*' $O/cfg_${c}_b$B.json)"
done
fi
if [ "${PART:-2}" = 2 ]; then
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > $O/layers_b512.txt 2>&1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run --output-format csv -- \
   python3 $R/bench.py --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/$O/prof_default.log 2>&1)
for spec in ssd:64 posenet:64 deeplab:8; do
  c=${spec%%:*}; B=${spec##*:}
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_${c}_b$B -o run --output-format csv -- \
     python3 $R/bench.py --config $c --batch $B --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/$O/prof_${c}_b$B.log 2>&1)
done
fi
echo done
