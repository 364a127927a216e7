"""hipBLASLt path numerics probe (pw_conv shapes that take it)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

torch.manual_seed(0)
for M, K, N, act, use_res in [(4096, 128, 64, 0, False), (4096, 128, 64, 1, False), (4096, 128, 64, 0, True),
                              (6272, 320, 1280, 0, False), (6272, 320, 1280, 1, False)]:
    x = torch.randn(M, K, device="cuda")
    wt = torch.randn((N + 15) // 16 * 16, K, device="cuda") / K ** 0.5
    bias = torch.randn(wt.shape[0], device="cuda")
    res = torch.randn(M, N, device="cuda") if use_res else None
    y = torch.ops.nnsx.pw_conv(x, wt, bias, res, N, act, True)
    ref = x @ wt[:N].t()
    nob = ref.clone()
    ref = ref + bias[:N]
    if use_res:
        ref = ref + res
    if act == 1:
        ref = ref.clamp(0, 6)
    err = (y - ref).abs().max().item()
    print(f"M={M} K={K} N={N} act={act} res={use_res}: max err {err:.3g}; y[0,:4] {y[0, :4].tolist()} "
          f"ref {ref[0, :4].tolist()} nobias {nob[0, :4].tolist()} relu6(nobias) {nob[0, :4].clamp(0, 6).tolist()}")
