#!/bin/bash
# Round-6 GPU check: comm tests (forced one-rank RCCL rounds), the 14x14 irp kernel's
# accuracy gate, the load-time lowering tests, per-layer A/B (NNSX_IRP=0 / 1) at batch
# 512, then the default bench and the lowered-plain-model bench.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6check
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_rccl_ranks.py -x -q --timeout 120 --timeout-method thread > $O/comm_tests.txt 2>&1 || { tail -30 $O/comm_tests.txt; exit 1; }
tail -2 $O/comm_tests.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_irp.py tests/test_gpu_lowering.py -q --timeout 200 --timeout-method thread > $O/irp_low_tests.txt 2>&1 || true
tail -25 $O/irp_low_tests.txt
for f in 14,64,384,64,1 14,64,384,96,1 14,96,576,96,1; do
  NNSX_IR_ONLY=$f NNSX_IRP=0 timeout -k 10 120 python -u scripts/bench_ir_f32.py 512 2>&1 | grep -v amdgpu.ids >> $O/layers_irp0.txt
  NNSX_IR_ONLY=$f NNSX_IRP=1 timeout -k 10 120 python -u scripts/bench_ir_f32.py 512 2>&1 | grep -v amdgpu.ids >> $O/layers_irp1.txt
done
cat $O/layers_irp0.txt $O/layers_irp1.txt | grep fused
timeout -k 10 400 python bench.py --sweep "" > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-300
NNSX_IRP=0 timeout -k 10 400 python bench.py --sweep "" --latency-frames 0 > $O/bench_irp0.json 2> $O/bench_irp0.err
tail -1 $O/bench_irp0.json | cut -c1-200
timeout -k 10 400 python bench.py --engine lowered --sweep "" --latency-frames 0 > $O/bench_lowered.json 2> $O/bench_lowered.err
tail -1 $O/bench_lowered.json | cut -c1-200
