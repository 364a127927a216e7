#!/bin/bash
# same-box A/B of whole-pipeline variants: scripts/gpu_r6_ab.sh <out file> <rounds> "<variant>" ...
# (each variant: space-separated NNSX_* settings or NONE=1); bench.py default config, 100 steps after 20
set -eo pipefail
cd "$(dirname "$0")/.."
out=$1; rounds=$2; shift 2
mkdir -p "$(dirname "$out")"
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    line=$(env $v timeout -k 10 300 python bench.py --sweep "" --latency-frames 0 2>/dev/null | tail -1)
    echo "$r [$v] $(echo "$line" | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"gpu_invoke_ms_median": [0-9.]*' | tr '\n' ' ')" | tee -a "$out"
  done
done
