"""Micro-benchmark: nnsx pw_gemm (torch.ops.nnsx.pw_conv) vs torch.matmul
(hipBLASLt) on the MobileNetV2 7x7 / head / classifier GEMM shapes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
SHAPES = [(B * 49, 160, 960, 1), (B * 49, 960, 160, 0), (B * 49, 960, 320, 0), (B * 49, 320, 1280, 1),
          (B, 1280, 1000, 0), (B * 196, 96, 576, 1), (B * 196, 576, 96, 0), (B * 3136, 24, 144, 1)]


def timeit(fn, n=30):
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
    kp = (K + 31) // 32 * 32
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    wt = torch.zeros((N + 63) // 64 * 64, kp, device="cuda", dtype=torch.bfloat16)
    wt[:N, :K] = torch.randn(N, K, device="cuda").to(torch.bfloat16) * 0.05
    bias = torch.zeros(wt.shape[0], device="cuda")
    out_f32 = M == B
    t_nnsx = timeit(lambda: torch.ops.nnsx.pw_conv(x.view(M, 1, 1, K), wt, bias, None, N, act, out_f32))
    w2 = wt[:N, :K].t().contiguous()
    t_blas = timeit(lambda: torch.matmul(x, w2))
    flops = 2.0 * M * K * N
    print(f"M={M:6d} K={K:4d} N={N:4d}: nnsx {t_nnsx:7.1f}us ({flops / t_nnsx / 1e6:6.1f} TF/s)   "
          f"hipBLASLt matmul {t_blas:7.1f}us ({flops / t_blas / 1e6:6.1f} TF/s)", flush=True)


DW = [(B, 112, 112, 96, 2), (B, 56, 56, 144, 1), (B, 14, 14, 576, 1), (B, 7, 7, 960, 1)]
for b, h, w_, c, st in DW:
    x = torch.randn(b, h, w_, c, device="cuda").to(torch.bfloat16)
    wd = (torch.randn(9, c, device="cuda") * 0.1).to(torch.bfloat16)
    bd = torch.zeros(c, device="cuda")
    t = timeit(lambda: torch.ops.nnsx.dw_conv(x, wd, bd, st, 1))
    nbytes = x.numel() * 2 * (1 + 1 / (st * st))
    print(f"dw3x3 {b}x{h}x{w_}x{c} s{st}: {t:7.1f}us ({nbytes / t / 1e6:6.2f} TB/s)", flush=True)
