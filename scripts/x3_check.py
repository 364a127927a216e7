"""Quick x3 GEMM correctness probe: max |err| vs fp64 for a few shapes / tiles
(the package is imported from the directory given as argv[1], default: repo)."""
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, root)
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

print("package", nnstreamer_amd.__file__)
torch.ops.nnsx.set_f32_math("x3")
for M, K, N in [(1000, 16, 96), (777, 24, 144), (6272, 960, 320), (130, 1280, 1000), (4225, 64, 128)]:
    for tile in (0, 64064, 128064, 64128):
        for cache in (True, False):
            torch.ops.nnsx.x3_weight_cache(cache)
            torch.manual_seed(M + K)
            x = (torch.randn(M, K, device="cuda") * 2).clamp(0, 6)
            npad, kpad = (N + 15) // 16 * 16, (K + 7) // 8 * 8
            wt = torch.zeros(npad, kpad, device="cuda")
            wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
            b = torch.randn(npad, device="cuda")
            y = torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, None, N, 0, tile)
            ref = x.double() @ wt[:N, :K].double().t() + b[:N].double()
            print(f"{M:6d} {K:5d} {N:5d} tile {tile:6d} w3 {int(cache)}  max err {(y.double() - ref).abs().max().item():.3e}")
