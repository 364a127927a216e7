#!/bin/bash
# board power and gfx clock while bench.py runs a sustained 600-step pass, per variant:
#   scripts/gpu_r6_powmon.sh <outdir> "<variant>" ...
set -eo pipefail
cd "$(dirname "$0")/.."
O=$1; shift
mkdir -p $O
for v in "$@"; do
  tag=$(echo "$v" | tr ' =' '__')
  env $v timeout -k 10 300 python bench.py --sweep "" --latency-frames 0 --steps 600 --warmup 20 > $O/$tag.json 2> $O/$tag.err &
  pid=$!
  : > $O/$tag.smi
  while kill -0 $pid 2>/dev/null; do
    timeout -k 2 5 amd-smi metric -p -c -g 0 --csv >> $O/$tag.smi 2>&1 || true
    sleep 0.2
  done
  wait $pid
  echo "[$v] $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/$tag.json | tr '\n' ' ')"
done
