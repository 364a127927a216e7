#!/bin/bash
# Round 4: small-batch forward traces (batch 1 and 8: back-to-back graph replays)
# and the ATen-origin analysis of a short bench run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for B in 1 8; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fwdprof_b$B -o fwd --output-format csv -- python3 $R/scripts/b1_graph_probe.py $B > $R/gpurun_out/fwdprof_b$B.log 2>&1 || { echo "fwd prof $B failed"; tail -20 $R/gpurun_out/fwdprof_b$B.log; exit 1; }
  grep -E "graph replay" $R/gpurun_out/fwdprof_b$B.log
done
# padded-frame upload micro-bench (DeepLab 513 / PoseNet 257 wide): DMA + unpad vs the gather kernel
cd $R && for w in 513:8 257:64; do
  timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 && \
  NNSX_CONVERTER_PADDED_DMA=0 timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 || { echo "upload bench failed"; tail -20 gpurun_out/upload_bench.txt; exit 1; }
done
cat gpurun_out/upload_bench.txt
# batch 8 as the headline run (long window): pipeline ms per batch vs device ms per invoke
# (replay lanes: auto = 2 at these batches, NNSX_TORCH_LANES=1 the single-stream A/B)
cd $R && for B in 8 32; do for L in 1 0 3; do
  NNSX_TORCH_LANES=$L timeout -k 10 300 python3 bench.py --batch $B --steps 400 --warmup 20 --latency-frames 0 --sweep "" > gpurun_out/bench_b${B}_l$L.log 2>&1 || { echo "bench b$B lanes $L failed"; tail -20 gpurun_out/bench_b${B}_l$L.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bench_b${B}_l$L.log') if l.startswith('{')][-1]); print('b$B lanes=$L', d['value'], d['ms_per_step'], d['gpu_invoke_ms_median'], d['p50_latency_ms'])"
done; done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_aten -o aten -- python3 $R/bench.py --steps 10 --warmup 3 --latency-frames 50 --sweep 8 > $R/gpurun_out/prof_aten.log 2>&1 || { echo "aten prof failed"; tail -20 $R/gpurun_out/prof_aten.log; exit 1; }
cd $R && python3 scripts/aten_origin.py gpurun_out/prof_aten/aten_results.db > gpurun_out/aten_origin.txt 2>&1; tail -30 gpurun_out/aten_origin.txt
