#!/bin/bash
# configs 3-5 at bench.py's default batch (512 frames per invoke)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/b512cfg.txt
: > $out
for c in ssd deeplab posenet; do
  timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 5 --sweep "" --latency-frames 0 > gpurun_out/b512_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/b512_$c.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/b512_$c.log') if l.startswith('{')][-1]); print('$c', d['config'].get('global_batch'), d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))" | tee -a $out
done
