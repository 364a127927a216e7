#!/bin/bash
# Round 4: upload micro-bench (host reference, DMA, split DMA) and the replay-lane A/B
# at batch 8 / 16 / 32 (subset of gpu_r4_small.sh, without the traces).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
# padded-frame upload micro-bench (DeepLab 513 / PoseNet 257 wide): DMA + unpad vs the gather kernel
rm -f gpurun_out/upload_bench.txt
cd $R && for w in 513:8 257:64; do
  UPLOAD_BENCH_HOST=1 timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 && \
  timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 && \
  NNSX_CONVERTER_DMA_SPLIT=2 timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 && \
  NNSX_CONVERTER_DMA_SPLIT=4 timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 || { echo "upload bench failed"; tail -20 gpurun_out/upload_bench.txt; exit 1; }
done
cat gpurun_out/upload_bench.txt
# batch 8 as the headline run (long window): pipeline ms per batch vs device ms per invoke
# (replay lanes: auto = 2 at these batches, NNSX_TORCH_LANES=1 the single-stream A/B)
cd $R && for B in 8 16 32; do for L in 1 2 3 4; do
  NNSX_TORCH_LANES=$L timeout -k 10 300 python3 bench.py --batch $B --steps 400 --warmup 20 --latency-frames 0 --sweep "" > gpurun_out/bench_b${B}_l$L.log 2>&1 || { echo "bench b$B lanes $L failed"; tail -20 gpurun_out/bench_b${B}_l$L.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bench_b${B}_l$L.log') if l.startswith('{')][-1]); print('b$B lanes=$L', d['value'], d['ms_per_step'], d['gpu_invoke_ms_median'], d['p50_latency_ms'])"
done; done
