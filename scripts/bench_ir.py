"""Micro-benchmark: fused ir_block vs the unfused pw->dw->pw chain for every
MobileNetV2 block shape at batch B (GPU time via CUDA events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
SHAPES = [(112, 32, 32, 16, 1), (112, 16, 96, 24, 2), (56, 24, 144, 24, 1), (56, 24, 144, 32, 2),
          (28, 32, 192, 32, 1), (28, 32, 192, 64, 2), (14, 64, 384, 64, 1), (14, 64, 384, 96, 1),
          (14, 96, 576, 96, 1), (14, 96, 576, 160, 2), (7, 160, 960, 160, 1), (7, 160, 960, 320, 1)]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


ONLY = os.environ.get("NNSX_IR_ONLY")  # e.g. "56,24,144,24,1": one shape, fused only (for rocprof)
if ONLY:
    SHAPES = [tuple(int(v) for v in ONLY.split(","))]
tot_f = tot_u = 0.0
for H, cin, hid, cout, st in SHAPES:
    has_expand = not (cin == 32 and hid == 32)
    hp = (hid + 31) // 32 * 32
    cin32 = (cin + 31) // 32 * 32
    x = torch.randn(B, H, H, cin, device="cuda").to(torch.bfloat16)
    we = (torch.randn((hp + 63) // 64 * 64, cin32, device="cuda") * 0.1).to(torch.bfloat16)
    be = torch.zeros(we.shape[0], device="cuda")
    wd = (torch.randn(9, hp, device="cuda") * 0.3).to(torch.bfloat16)
    bd = torch.zeros(hp, device="cuda")
    wp = (torch.randn((cout + 63) // 64 * 64, hp, device="cuda") * 0.1).to(torch.bfloat16)
    bp = torch.zeros(wp.shape[0], device="cuda")
    res = st == 1 and cin == cout
    ok = torch.ops.nnsx.ir_supported(st, cin, hp, cout)

    def unf():
        h = torch.ops.nnsx.pw_conv(x, we, be, None, hp, 1, False) if has_expand else x
        h = torch.ops.nnsx.dw_conv(h, wd, bd, st, 1)
        return torch.ops.nnsx.pw_conv(h, wp, bp, x if res else None, cout, 0, False)

    tu = timeit(unf) if not ONLY else 0.0
    tf = timeit(lambda: torch.ops.nnsx.ir_block(x, we[:hp].contiguous(), be[:hp].contiguous(), wd, bd, wp, bp, st,
                                                cout, has_expand, res)) if ok else float("nan")
    nbytes = (x.numel() + B * ((H - 1) // st + 1) ** 2 * cout) * 2
    tot_u += tu
    tot_f += tf if ok else tu
    print(f"H={H:3d} {cin:3d}->{hid:3d}->{cout:3d} s{st}: unfused {tu:8.1f}us  fused {tf:8.1f}us  "
          f"(fused io {nbytes / tf / 1e6 if ok else 0:6.2f} TB/s)", flush=True)
print(f"total unfused {tot_u:.1f}us  fused(best-available) {tot_f:.1f}us")
