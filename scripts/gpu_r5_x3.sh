#!/bin/bash
# round 5: split-bf16 (x3) tests + per-block and whole-model A/B
cd "$(dirname "$0")/.."
NNSX_X3_IRW=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py -q --timeout 120 --timeout-method thread > gpurun_out/x3_tests.txt 2>&1
tail -3 gpurun_out/x3_tests.txt
NNSX_X3_IRW=1 timeout -k 10 240 python -u scripts/x3_blocks_ab.py 512 3 > gpurun_out/x3_blocks.txt 2>&1 || exit 1
NNSX_X3_IRW=1 timeout -k 10 300 python -u scripts/x3_ab.py --rounds 3 --skip-gemm > gpurun_out/x3_model.txt 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode_stage.py -q --timeout 120 --timeout-method thread > gpurun_out/decode_stage.txt 2>&1
tail -3 gpurun_out/decode_stage.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_memcheck.py -q --timeout 300 --timeout-method thread > gpurun_out/memcheck.txt 2>&1
tail -3 gpurun_out/memcheck.txt
