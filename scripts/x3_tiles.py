"""x3 GEMM tile sweep (pw_conv_f32_tile: 64x64, 128x64, 64x128, 128x128) vs the
auto tile of both methods, on the benched GEMM shapes.  Median us of R rounds."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

SHAPES = [(512 * 49, 960, 320), (512 * 49, 320, 1280), (64 * 65 * 65, 128, 128), (64 * 33 * 33, 256, 256),
          (64 * 17 * 17, 512, 512), (64 * 17 * 17, 1024, 1024), (512 * 196, 96, 576), (8 * 33 * 33, 320, 256)]


def timeit(fn, n=20):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


R = 3
print(f"{'M':>7s} {'K':>5s} {'N':>5s} | fp32 auto | x3 auto  64x64  128x64  64x128 128x128 | best x3 TF/s")
for M, K, N in SHAPES:
    x = (torch.randn(M, K, device="cuda") * 2).clamp(0, 6)
    npad, kpad = (N + 15) // 16 * 16, (K + 7) // 8 * 8
    wt = torch.zeros(npad, kpad, device="cuda")
    wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
    b = torch.zeros(npad, device="cuda")
    cases = {"fp32": ("fp32", 0), "x3": ("x3", 0)}
    for t in (64064, 128064, 64128, 128128):
        cases[str(t)] = ("x3", t)
    res = {k: [] for k in cases}
    for _ in range(R):
        for k, (m, t) in cases.items():
            torch.ops.nnsx.set_f32_math(m)
            if t:
                res[k].append(timeit(lambda: torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, None, N, 1, t)))
            else:
                res[k].append(timeit(lambda: torch.ops.nnsx.pw_conv(x, wt, b, None, N, 1, True)))
    med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
    best = min(med[k] for k in ("64064", "128064", "64128", "128128"))
    print(f"{M:7d} {K:5d} {N:5d} | {med['fp32']:8.1f} | {med['x3']:7.1f} {med['64064']:6.1f} {med['128064']:7.1f} "
          f"{med['64128']:7.1f} {med['128128']:7.1f} | {2 * M * K * N / best / 1e6:6.1f}", flush=True)
