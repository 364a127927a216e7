"""Batch-1 launch-path probe of the fp32 fused MobileNetV2: host time of a
hipGraph replay vs. eager launches, and replay->sync latency (no profiler).

    python scripts/b1_graph_probe.py [batch]     (default 1)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402
from nnstreamer_amd.models.fused import fused_mobilenet_v2  # noqa: E402

m = torch.jit.script(fused_mobilenet_v2(0, "fp32").cuda())
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
x = torch.randint(0, 256, (B, 224, 224, 3), device="cuda", dtype=torch.uint8)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(5):
        m(x)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    y = m(x)
torch.cuda.synchronize()


def probe(fn, n=200):
    host, e2e = [], []
    for _ in range(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        host.append((t1 - t0) * 1e6)
        e2e.append((t2 - t0) * 1e6)
    host.sort()
    e2e.sort()
    return host[n // 2], e2e[n // 2], e2e[int(n * 0.99)]


for name, fn in [("graph replay", g.replay), ("eager forward", lambda: m(x))]:
    h, e, e99 = probe(fn)
    print(f"{name:14s} host {h:7.1f} us   launch->sync p50 {e:7.1f} us  p99 {e99:7.1f} us", flush=True)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
ev0.record()
for _ in range(100):
    g.replay()
ev1.record()
torch.cuda.synchronize()
print(f"batch {B}: graph replay back-to-back: {ev0.elapsed_time(ev1) * 10:.1f} us per forward (device)")
