"""CPU cost of replaying a captured fused model (python-side torch.cuda.graph),
to separate model launch cost from pipeline effects."""
import sys
import time

import torch

sys.path.insert(0, ".")
import nnstreamer_amd  # noqa: F401  (loads the ops)
from nnstreamer_amd.models.export import build_model

name, S, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
m = torch.jit.freeze(torch.jit.script(build_model(name).cuda().eval()))
x = torch.randint(0, 255, (B, S, S, 3), dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
with torch.inference_mode():
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            m(x)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        m(x)
    te = (time.perf_counter() - t) / 10 * 1e3
    torch.cuda.synchronize()
    te2 = (time.perf_counter() - t) / 10 * 1e3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m(x)
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        g.replay()
    tg = (time.perf_counter() - t) / 10 * 1e3
    torch.cuda.synchronize()
    tg2 = (time.perf_counter() - t) / 10 * 1e3
print(f"{name} B={B}: eager CPU {te:.2f} ms (wall {te2:.2f}); graph replay CPU {tg:.2f} ms (wall {tg2:.2f})")
