"""One fp32 GEMM shape run R times (for rocprofv3 --pmc passes): method
(x3 | fp32) and tile from the command line.

    python scripts/gemm_one.py M K N [method] [tile] [R]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

M, K, N = (int(v) for v in sys.argv[1:4])
method = sys.argv[4] if len(sys.argv) > 4 else "x3"
tile = int(sys.argv[5]) if len(sys.argv) > 5 else 0
R = int(sys.argv[6]) if len(sys.argv) > 6 else 10
torch.ops.nnsx.set_f32_math(method)
torch.manual_seed(0)
x = (torch.randn(M, K, device="cuda") * 2).clamp(0, 6)
npad, kpad = (N + 15) // 16 * 16, (K + 7) // 8 * 8
wt = torch.zeros(npad, kpad, device="cuda")
wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
b = torch.randn(npad, device="cuda")
for _ in range(R):
    torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, None, N, 1, tile)
torch.cuda.synchronize()
print("done", M, K, N, method, tile)
