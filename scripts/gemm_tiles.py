"""fp32 GEMM tile A/B (nnsx::pw_conv_f32_tile) on the MobileNetV2 batch-512 chain shapes: us per call per tile."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

SHAPES = [(25088, 960, 320, 0), (25088, 160, 960, 1), (25088, 320, 1280, 1), (6272, 960, 320, 0), (5184, 512, 1024, 1),
          (5184, 1024, 1024, 1), (18496, 512, 512, 1)]
TILES = [0, 64064, 128064, 64128, 128128, 128192]


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


for M, K, N, act in SHAPES:
    x = torch.randn(M, K, device="cuda")
    wt = torch.randn((N + 63) // 64 * 64, K, device="cuda") / K ** 0.5
    b = torch.randn(wt.shape[0], device="cuda")
    ref = torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, None, N, act, 64064)
    row = []
    for t in TILES:
        y = torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, None, N, act, t)
        assert (y - ref).abs().max().item() < 1e-3
        row.append(f"{t}:{timeit(lambda: torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, None, N, act, t)):7.1f}")
    print(f"M={M:6d} K={K:5d} N={N:5d} act={act}  " + "  ".join(row), flush=True)
