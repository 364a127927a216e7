#!/bin/bash
# Round 4: the whole GPU test suite, smoke(), the default bench (driver's command), H2D link probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_full.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_full.log; exit 1; }
tail -3 gpurun_out/pytest_full.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
timeout -k 10 60 python3 -c "
import torch, time
for mb in (64, 256):
    h = torch.empty(mb << 20, dtype=torch.uint8).pin_memory(); d = torch.empty_like(h, device='cuda')
    for _ in range(3): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(10): d.copy_(h, non_blocking=True)
    torch.cuda.synchronize(); el = time.perf_counter() - t
    print(f'H2D pinned {mb} MB: {10 * mb / 1024 / el:.1f} GB/s')
"
