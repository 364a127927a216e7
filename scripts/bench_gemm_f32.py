"""fp32 pointwise GEMM: nnsx pw_conv (MFMA 16x16x4 f32, bias + ReLU6 fused)
vs torch.addmm + clamp (hipBLASLt / rocBLAS fp32) on the PoseNet (MobileNetV1
257, batch 64) and MobileNetV2 head shapes.  Prints us per call and TF/s."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

torch.backends.cuda.matmul.allow_tf32 = False
SHAPES = [  # (M, K, N)
    (64 * 65 * 65, 64, 128), (64 * 65 * 65, 128, 128), (64 * 33 * 33, 128, 256), (64 * 33 * 33, 256, 256),
    (64 * 17 * 17, 256, 512), (64 * 17 * 17, 512, 512), (64 * 17 * 17, 512, 1024), (64 * 17 * 17, 1024, 1024),
    (512 * 49, 320, 1280), (512 * 49, 960, 320),
]


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


for M, K, N in SHAPES:
    x = torch.randn(M, K, device="cuda")
    w = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.randn(N, device="cuda")
    npad, kpad = (N + 15) // 16 * 16, (K + 7) // 8 * 8
    wt = torch.zeros(npad, kpad, device="cuda")
    wt[:N, :K] = w
    bp = torch.zeros(npad, device="cuda")
    bp[:N] = b
    wT = w.t().contiguous()
    us_n = timeit(lambda: torch.ops.nnsx.pw_conv(x, wt, bp, None, N, 1, True))
    us_t = timeit(lambda: torch.addmm(b, x, wT).clamp_(0, 6))
    us_m = timeit(lambda: torch.mm(x, wT))
    fl = 2.0 * M * K * N
    print(f"M={M:7d} K={K:5d} N={N:5d}  nnsx {us_n:8.1f} us {fl / us_n / 1e6:6.1f} TF/s | torch addmm+clamp {us_t:8.1f} us "
          f"| mm only {us_m:8.1f} us {fl / us_m / 1e6:6.1f} TF/s")
