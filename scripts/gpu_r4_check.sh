#!/bin/bash
# Round-4 GPU session: full GPU tests, smoke, bench, and a kernel trace of the
# forced-RCCL group-of-one test (shows the RCCL kernels executing on one GPU).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_round.sh test && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log && \
timeout -k 10 400 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && cut -c1-400 gpurun_out/bench_default.json && \
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_rccl1 -o rccl1 -- \
   python -m pytest $GRAFT_REPO_ROOT/tests/test_gpu_comm.py -k forced_rccl -q -p no:cacheprovider > $GRAFT_REPO_ROOT/gpurun_out/prof_rccl1.log 2>&1) && \
tail -3 gpurun_out/prof_rccl1.log
