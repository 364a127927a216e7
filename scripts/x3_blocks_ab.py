"""Per-block A/B of the fp32 engine's product method on MobileNetV2's fused
inverted residuals at batch B: native fp32 MFMA (irw_f32) vs split-bf16
(irw_x3), interleaved rounds in one process, median us per block.

    python scripts/x3_blocks_ab.py [B] [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402
from nnstreamer_amd.models.fused import x3_split  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
R = int(sys.argv[2]) if len(sys.argv) > 2 else 5
PEAK = 157.3e12
SHAPES = [(112, 16, 96, 24, 2), (56, 24, 144, 24, 1), (56, 24, 144, 32, 2), (28, 32, 192, 32, 1),
          (28, 32, 192, 64, 2), (14, 64, 384, 64, 1), (14, 64, 384, 96, 1), (14, 96, 576, 96, 1),
          (14, 96, 576, 160, 2), (7, 160, 960, 160, 1), (7, 160, 960, 320, 1)]
COUNT = {(28, 32, 192, 32, 1): 2, (14, 64, 384, 64, 1): 3, (14, 96, 576, 96, 1): 2, (7, 160, 960, 160, 1): 2}


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


print(f"# fused inverted residuals, batch {B}, median of {R} interleaved rounds (us); x count = blocks in MobileNetV2")
tot = {"fp32": 0.0, "x3": 0.0}
for H, cin, hid, cout, st in SHAPES:
    torch.manual_seed(H + cin + hid)
    kin = (cin + 7) // 8 * 8
    x = (torch.randn(B, H, H, cin, device="cuda"))
    we = torch.zeros(hid, kin, device="cuda")
    we[:, :cin] = torch.randn(hid, cin, device="cuda") / cin ** 0.5
    be = torch.randn(hid, device="cuda") * 0.1
    wd = torch.randn(9, hid, device="cuda") / 3
    bd = torch.randn(hid, device="cuda") * 0.1
    npad = (cout + 15) // 16 * 16
    wp = torch.zeros(npad, hid, device="cuda")
    wp[:cout] = torch.randn(cout, hid, device="cuda") / hid ** 0.5
    bp = torch.zeros(npad, device="cuda")
    we3 = x3_split(we[:, :cin].cpu(), hid, (cin + 31) // 32 * 32).cuda()
    wp3 = x3_split(wp[:cout].cpu(), (cout + 31) // 32 * 32, hid).cuda()
    res = st == 1 and cin == cout
    tk = torch.zeros(768, dtype=torch.int32, device="cuda")
    if torch.ops.nnsx.ir_supported_f32(st, H, H, cin, hid, cout, True):
        def fn():
            return torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, st, cout, True, res, 1, tk, we3, wp3)
        tag = "fused"
    else:
        def fn():
            h = torch.ops.nnsx.ir_expand_dw(x, we, be, wd, bd, st, 1, we3)
            return torch.ops.nnsx.pw_conv(h, wp, bp, x if res else None, cout, 0, True)
        tag = "exp+dw,GEMM"
    t = {"fp32": [], "x3": []}
    meth = {}
    for _ in range(R):
        for m in ("fp32", "x3"):
            torch.ops.nnsx.set_f32_math(m)
            meth[m] = torch.ops.nnsx.ir_method_f32(st, H, H, cin, hid, cout, B, 1)
            t[m].append(timeit(fn))
    med = {m: sorted(v)[len(v) // 2] for m, v in t.items()}
    n = COUNT.get((H, cin, hid, cout, st), 1)
    for m in med:
        tot[m] += n * med[m]
    Ho = (H - 1) // st + 1
    flop = 2 * B * (H * H * cin * hid + Ho * Ho * hid * 9 + Ho * Ho * hid * cout)
    print(f"{tag:11s} H={H:3d} {cin:3d}->{hid:3d}->{cout:3d} s{st} x{n}  fp32 {med['fp32']:7.1f}  "
          f"x3 {med['x3']:7.1f} ({meth['x3']:4s})  {med['fp32'] / med['x3']:5.2f}x  "
          f"[{flop / med['x3'] / 1e6:6.1f} TF/s-equiv]", flush=True)
print(f"blocks total (with repeats): fp32 {tot['fp32']:.0f} us, x3 {tot['x3']:.0f} us")
