"""fp32 (x3) GEMM tile A/B on the configs-3..5 shapes whose 128 x 64 grid is
under one workgroup per CU: us per call for each tile, residual as in the model.

    python scripts/gemm_fill.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

# (label, M, K, N, act, residual)
SHAPES = [
    ("deeplab b8 project 960->160 +res", 8712, 960, 160, 0, True),
    ("deeplab b8 project 960->320", 8712, 960, 320, 0, False),
    ("deeplab b8 project 576->160", 8712, 576, 160, 0, False),
    ("deeplab b8 expand 160->960", 8712, 160, 960, 1, False),
    ("deeplab b8 aspp 320->256", 8712, 320, 256, 1, False),
    ("ssd b64 extra 1280->256", 6400, 1280, 256, 1, False),
    ("ssd b64 head 320->1280", 6400, 320, 1280, 1, False),
    ("mbv2 b512 7x7 project 960->320", 25088, 960, 320, 0, False),
    ("mbv2 b512 7x7 project 960->160 +res", 25088, 960, 160, 0, True),
    ("posenet b64 9x9 1024->1024", 5184, 1024, 1024, 1, False),
    ("posenet b64 9x9 512->1024", 5184, 512, 1024, 1, False),
    ("posenet b64 17x17 512->512", 18496, 512, 512, 1, False),
    ("mbv2 b512 classifier 1280->1000", 512, 1280, 1000, 0, False),
    ("mbv2 b512 head 320->1280", 25088, 320, 1280, 1, False),
]
TILES = [int(t) for t in os.environ.get("TILES", "0,64064,128064").split(",")]


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


torch.manual_seed(0)
for label, M, K, N, act, has_res in SHAPES:
    x = (torch.randn(M, K, device="cuda") * 2).clamp(0, 6)
    wt = torch.zeros((N + 63) // 64 * 64, (K + 31) // 32 * 32, device="cuda")
    wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(wt.shape[0], device="cuda")
    r = torch.randn(M, N, device="cuda") if has_res else None
    ref = torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, r, N, act, 64064)
    row = []
    for t in TILES:
        y = torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, r, N, act, t)
        assert (y - ref).abs().max().item() < 1e-3, (label, t)
        row.append(f"{t}:{timeit(lambda: torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, r, N, act, t)):7.1f}")
    print(f"{label:38s} M={M:6d} K={K:5d} N={N:5d}  " + "  ".join(row), flush=True)
