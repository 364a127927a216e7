#!/bin/bash
# A/B of a code-generation variant (variants/$V: a copy of the package built with other hipcc flags)
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
V=${V:-vf}
timeout -k 10 300 python -u scripts/x3_tiles.py > gpurun_out/ab_tiles_base.txt 2>&1
timeout -k 10 300 python -u variants/$V/scripts/x3_tiles.py > gpurun_out/ab_tiles_$V.txt 2>&1
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > gpurun_out/ab_layers_base.txt 2>&1
timeout -k 10 300 python -u variants/$V/scripts/bench_ir_f32.py 512 > gpurun_out/ab_layers_$V.txt 2>&1
for i in 1 2; do
timeout -k 10 300 python bench.py --sweep "" --latency-frames 0 > gpurun_out/ab_bench_base$i.json 2>/dev/null
timeout -k 10 300 python variants/$V/bench.py --sweep "" --latency-frames 0 > gpurun_out/ab_bench_$V$i.json 2>/dev/null
done
grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ab_bench_*.json
