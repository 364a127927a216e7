"""Depthwise 3x3 fp32 (nnsx::dw_conv, dw3x3_f32_col_kernel) against a plain device copy of the
same bytes (read input + write output), on the PoseNet / MobileNetV2 shapes.  Prints us per call and
the effective HBM rate of each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

SHAPES = [(64, 129, 32, 1, 1), (64, 129, 64, 2, 1), (64, 65, 128, 1, 1), (64, 33, 256, 1, 1), (64, 17, 512, 1, 1),
          (512, 7, 960, 1, 1), (512, 14, 576, 1, 1), (8, 33, 576, 1, 2), (8, 33, 960, 1, 2), (32, 33, 960, 1, 2)]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for B, H, C, S, D in SHAPES:
    x = torch.rand(B, H, H, C, device="cuda")
    w = torch.randn(9, C, device="cuda")
    b = torch.randn(C, device="cuda")
    y = torch.ops.nnsx.dw_conv(x, w, b, S, 1, D)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).double(), w.t().reshape(C, 1, 3, 3).double(), b.double(),
                                     stride=S, padding=D, dilation=D, groups=C).clamp(0, 6).permute(0, 2, 3, 1)
    err = ((y.double() - ref).abs() / (ref.abs() + 1)).max().item()
    assert err < 1e-5, err
    byt = x.numel() * 4 + y.numel() * 4
    us = timeit(lambda: torch.ops.nnsx.dw_conv(x, w, b, S, 1, D))
    xc = torch.empty_like(x)
    us_c = timeit(lambda: xc.copy_(x))
    print(f"B={B:4d} H={H:4d} C={C:5d} s{S} d{D}: dw {us:7.1f} us {byt / us / 1e6:5.2f} TB/s | copy of the input "
          f"{us_c:7.1f} us {2 * x.numel() * 4 / us_c / 1e6:5.2f} TB/s")
