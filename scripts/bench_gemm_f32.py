"""fp32 GEMM tile sweep (torch.ops.nnsx.pw_conv_f32_tile) over the MobileNetV2
1x1-conv shapes at batch B, plus the depthwise kernel variants."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
PEAK = 157.3e12
TILES = [64064, 128064, 64128, 128128, 128192, 0]
# (name, M, K, N, act)
SHAPES = [("e112 16->96", B * 112 * 112, 16, 96, 1), ("p56 96->24", B * 56 * 56, 96, 24, 0),
          ("e56 24->144", B * 56 * 56, 24, 144, 1), ("p56 144->24", B * 56 * 56, 144, 24, 0),
          ("e28 32->192", B * 28 * 28, 32, 192, 1), ("p28 192->32", B * 28 * 28, 192, 32, 0),
          ("e14 64->384", B * 196, 64, 384, 1), ("p14 384->64", B * 196, 384, 64, 0),
          ("p14 384->96", B * 196, 384, 96, 0), ("e14 96->576", B * 196, 96, 576, 1),
          ("p14 576->96", B * 196, 576, 96, 0), ("p7 576->160", B * 49, 576, 160, 0),
          ("e7 160->960", B * 49, 160, 960, 1), ("p7 960->160", B * 49, 960, 160, 0),
          ("p7 960->320", B * 49, 960, 320, 0), ("head 320->1280", B * 49, 320, 1280, 1),
          ("fc 1280->1000", B, 1280, 1000, 0), ("sq4096", 4096, 4096, 4096, 0)]


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


print("shape".ljust(18) + "".join(f"{t:>10d}" for t in TILES) + "   (us; 0 = auto)   best%peak")
for name, M, K, N, act in SHAPES:
    x = torch.randn(M, K, device="cuda")
    npad, kpad = (N + 15) // 16 * 16, (K + 7) // 8 * 8
    wt = torch.randn(npad, kpad, device="cuda") * 0.05
    bias = torch.zeros(npad, device="cuda")
    ref = None
    row = []
    for t in TILES:
        y = torch.ops.nnsx.pw_conv_f32_tile(x, wt, bias, None, N, act, t)
        if ref is None:
            ref = y
        else:
            assert torch.allclose(y, ref, rtol=1e-4, atol=1e-4), (name, t)
        row.append(timeit(lambda: torch.ops.nnsx.pw_conv_f32_tile(x, wt, bias, None, N, act, t)))
    fl = 2.0 * M * N * K
    print(name.ljust(18) + "".join(f"{u:10.1f}" for u in row) + f"   {100 * fl / min(row) / 1e-6 / PEAK:6.1f}%",
          flush=True)

for H, C, st in [(112, 96, 2), (56, 144, 1), (56, 144, 2), (28, 192, 1), (28, 192, 2), (14, 384, 1), (14, 576, 1),
                 (14, 576, 2), (7, 960, 1)]:
    x = torch.randn(B, H, H, C, device="cuda")
    w = torch.randn(9, C, device="cuda")
    b = torch.zeros(C, device="cuda")
    us = timeit(lambda: torch.ops.nnsx.dw_conv(x, w, b, st, 1, 1))
    ho = (H - 1) // st + 1
    nbytes = 4 * B * C * (H * H + ho * ho)
    print(f"dw H={H} C={C} s{st}: {us:8.1f} us  {nbytes / us / 1e6:6.2f} TB/s", flush=True)
