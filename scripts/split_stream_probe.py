"""Does splitting one batch into k independent sub-batches on k streams (k
parallel branches of one hipGraph) beat one stream at the same total batch?
Parallel branches let one branch's kernels fill the other's tail waves.

    python scripts/split_stream_probe.py [B] [precision]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402
from nnstreamer_amd.models.fused import fused_mobilenet_v2  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
m = torch.jit.script(fused_mobilenet_v2(0, prec).cuda())
x = torch.randint(0, 256, (B, 224, 224, 3), device="cuda", dtype=torch.uint8)


def build(k):
    streams = [torch.cuda.Stream() for _ in range(k)]
    parts = list(x.chunk(k))
    with torch.cuda.stream(streams[0]):
        for _ in range(3):
            for p in parts:
                m(p)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    outs = []
    with torch.cuda.graph(g, stream=streams[0]):
        main = torch.cuda.current_stream()
        for i, p in enumerate(parts):
            s = streams[i] if i else main
            if i:
                s.wait_stream(main)
            with torch.cuda.stream(s):
                outs.append(m(p))
        for s in streams[1:]:
            main.wait_stream(s)
    torch.cuda.synchronize()
    return g, outs


ref = None
for k in (1, 2, 4):
    g, outs = build(k)
    g.replay()
    torch.cuda.synchronize()
    y = torch.cat(outs)
    if ref is None:
        ref = y.clone()
    same = bool(torch.equal(y, ref))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(5):
        g.replay()
    e0.record()
    n = 50
    for _ in range(n):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"{prec} B={B} streams={k}: {ms * 1e3:8.1f} us per batch  {B / ms * 1e3:9.0f} frames/s  "
          f"bit-identical to 1 stream: {same}", flush=True)
