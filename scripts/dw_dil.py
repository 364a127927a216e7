"""Dilated depthwise (DeepLab's output-stride-16 maps) us per call: python scripts/dw_dil.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

for B, H, C in [(8, 33, 960), (8, 33, 576), (1, 33, 960), (1, 33, 576), (2, 33, 960), (32, 33, 960)]:
    x = torch.randn(B, H, H, C, device="cuda")
    w = torch.randn(9, C, device="cuda")
    b = torch.randn(C, device="cuda")
    for _ in range(5):
        torch.ops.nnsx.dw_conv(x, w, b, 1, 1, 2)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(50):
        torch.ops.nnsx.dw_conv(x, w, b, 1, 1, 2)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 50 * 1e3
    print(f"B={B:3d} {H}x{H}x{C:4d} dil 2: {us:7.1f} us  {2 * x.numel() * 4 / us / 1e6:5.2f} TB/s", flush=True)
