#!/bin/bash
# aligned-dword unpad_rows (HEAD tree) vs variants/base, same box
set -eo pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python -u -m pytest tests/test_gpu_elements.py -q -x --timeout 300 --timeout-method thread > gpurun_out/unpad_tests.txt 2>&1
grep -E "passed|failed" gpurun_out/unpad_tests.txt
for rep in 1 2 3; do
  for arm in new base; do
    b=bench.py; [ $arm = base ] && b=variants/base/bench.py
    timeout -k 10 300 python $b --config deeplab --batch 8 --sweep "" --latency-frames 0 > gpurun_out/unpad.json 2>/dev/null
    echo "$rep $arm deeplab b8 $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/unpad.json)"
  done
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ct_unpad -o run --output-format csv -- \
   python3 $R/bench.py --config deeplab --batch 8 --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/gpurun_out/ct_unpad.log 2>&1)
