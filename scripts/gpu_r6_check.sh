#!/bin/bash
# Round-6 quick GPU check: comm tests (forced one-rank RCCL rounds), then the default bench.
set -eo pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r6check
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_rccl_ranks.py -x -v --timeout 120 --timeout-method thread > $O/comm_tests.txt 2>&1
tail -3 $O/comm_tests.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-300
