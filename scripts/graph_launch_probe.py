"""Host cost of replaying the headline model's hipGraph: the fused fp32
MobileNetV2 at batch 512 captured with torch.cuda.CUDAGraph (what
tensor_filter custom=hipgraph:true replays), host microseconds per
graph.replay() call (no sync inside the timed call), device ms per replay, and
the number of kernels one replay runs.  Run it under different HIP runtime
settings (each in its own process) to see what the launch costs:

    python scripts/graph_launch_probe.py [batch]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402
from nnstreamer_amd.models.export import build_model  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    m = build_model("mobilenet_v2_fused_fp32", layout="nhwc").cuda().eval()
    x = torch.randn(B, 224, 224, 3, device="cuda")
    s = torch.cuda.Stream()
    with torch.no_grad():
        with torch.cuda.stream(s):
            for _ in range(3):
                m(x)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            y = m(x)
    torch.cuda.synchronize()
    host, dev = [], []
    for i in range(30):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t = time.perf_counter()
        g.replay()
        host.append((time.perf_counter() - t) * 1e6)
        e1.record()
        torch.cuda.synchronize()
        dev.append(e0.elapsed_time(e1))
    # back-to-back replays: host rate when the device is busy
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(10):
        g.replay()
    t_issue = (time.perf_counter() - t) * 1e6 / 10
    torch.cuda.synchronize()
    host.sort()
    dev.sort()
    env = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith(("DEBUG_", "HIP_", "AMD_")))
    print(f"[{env or 'defaults'}] B={B}: replay host us median {host[len(host) // 2]:.1f} (min {host[0]:.1f}), "
          f"back-to-back issue {t_issue:.1f} us/replay, device ms median {dev[len(dev) // 2]:.3f}; out {tuple(y.shape)}",
          flush=True)


if __name__ == "__main__":
    main()
