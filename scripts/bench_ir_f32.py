"""Micro-benchmark of the fp32 MobileNetV2 engine, layer by layer, at batch B:
every inverted-residual block (fused ir_block when supported, else the
pw -> dw -> pw chain), the stem, the head GEMM, pool and classifier.
Prints GPU time (CUDA events) and the fraction of the fp32 MFMA peak.

    python scripts/bench_ir_f32.py [B]          # NNSX_IR_ONLY=H,cin,hid,cout,s: one block (for rocprof)
                                                # NNSX_IR_ONLY=stem: the fused stem + block 1 only
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402
from nnstreamer_amd.models.fused import input_lut, x3_split  # noqa: E402

PEAK = 157.3e12
LUT = input_lut(-127.5, 127.5).cuda() if torch.cuda.is_available() else None
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
SHAPES = [(112, 32, 32, 16, 1), (112, 16, 96, 24, 2), (56, 24, 144, 24, 1), (56, 24, 144, 32, 2),
          (28, 32, 192, 32, 1), (28, 32, 192, 32, 1), (28, 32, 192, 64, 2), (14, 64, 384, 64, 1),
          (14, 64, 384, 64, 1), (14, 64, 384, 64, 1), (14, 64, 384, 96, 1), (14, 96, 576, 96, 1),
          (14, 96, 576, 96, 1), (14, 96, 576, 160, 2), (7, 160, 960, 160, 1), (7, 160, 960, 160, 1),
          (7, 160, 960, 320, 1)]


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


def row(name, us, flop):
    print(f"{name:34s} {us:8.1f} us  {flop / us / 1e6:7.1f} TF/s  {100 * flop / us / 1e-6 / PEAK:5.1f}% of fp32 peak",
          flush=True)


ONLY = os.environ.get("NNSX_IR_ONLY")
if ONLY == "stem":  # only the fused stem + block 1 (for rocprof)
    xu = torch.randint(0, 256, (B, 224, 224, 3), device="cuda", dtype=torch.uint8)
    w = [torch.randn(3, 3, 3, 32, device="cuda"), torch.zeros(32, device="cuda"), torch.randn(9, 32, device="cuda"),
         torch.zeros(32, device="cuda"), torch.randn(16, 32, device="cuda") * 0.1, torch.zeros(16, device="cuda")]
    us1 = timeit(lambda: torch.ops.nnsx.stem_ir1(xu, *w, LUT))
    print(f"stem+block1 fused ({ONLY}) {us1:.1f} us at batch {B}")
    sys.exit(0)
if ONLY:
    SHAPES = [tuple(int(v) for v in ONLY.split(","))]
total = 0.0
seen = {}
for H, cin, hid, cout, st in SHAPES:
    key = (H, cin, hid, cout, st)
    Ho = (H - 1) // st + 1
    flop = 2 * B * ((H * H * cin * hid if hid != cin else 0) + Ho * Ho * hid * 9 + Ho * Ho * hid * cout)
    if key in seen:
        total += seen[key]
        row(f"  (repeat) {key}", seen[key], flop)
        continue
    has_expand = hid != cin
    kin = (cin + 7) // 8 * 8
    x = torch.randn(B, H, H, cin, device="cuda")
    we = torch.randn(hid, kin, device="cuda") * 0.1
    be = torch.zeros(hid, device="cuda")
    wd = torch.randn(9, hid, device="cuda") * 0.3
    bd = torch.zeros(hid, device="cuda")
    npad = (cout + 15) // 16 * 16
    wp = torch.randn(npad, hid, device="cuda") * 0.1
    bp = torch.zeros(npad, device="cuda")
    res = st == 1 and cin == cout
    ok = bool(torch.ops.nnsx.ir_supported_f32(st, H, H, cin, hid, cout, has_expand))
    # split-bf16 weights: the x3 kernel runs when NNSX_F32_MATH (default x3) and NNSX_X3_IRW select it
    we3 = x3_split(we[:, :cin].cpu(), hid, (cin + 31) // 32 * 32).cuda() if has_expand else None
    wp3 = x3_split(wp[:cout].cpu(), (cout + 31) // 32 * 32, hid).cuda() if has_expand else None
    if ok:
        fn = lambda: torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, st, cout, has_expand, res, 1, None,  # noqa: E731
                                             we3, wp3)
        tag = "fused"
    elif has_expand and bool(torch.ops.nnsx.ir_expand_dw_supported_f32(st, H, H, cin, hid, B)):
        def fn():
            h = torch.ops.nnsx.ir_expand_dw(x, we, be, wd, bd, st)
            return torch.ops.nnsx.pw_conv(h, wp, bp, x if res else None, cout, 0, True)
        tag = "exp+dw, GEMM"
    else:
        def fn():
            h = torch.ops.nnsx.pw_conv(x, we, be, None, hid, 1, True) if has_expand else x
            h = torch.ops.nnsx.dw_conv(h, wd, bd, st, 1, 1)
            return torch.ops.nnsx.pw_conv(h, wp, bp, x if res else None, cout, 0, True)
        tag = "chain"
    us = timeit(fn)
    seen[key] = us
    total += us
    row(f"{tag} H={H} {cin}->{hid}->{cout} s{st}", us, flop)

if not ONLY:
    xu = torch.randint(0, 256, (B, 224, 224, 3), device="cuda", dtype=torch.uint8)
    ws = torch.randn(3, 3, 3, 32, device="cuda")
    bs = torch.zeros(32, device="cuda")
    us = timeit(lambda: torch.ops.nnsx.stem_conv_u8(xu, ws, bs, 1, LUT, True))
    total += us
    row("stem 224 u8 -> 32", us, 2 * B * 112 * 112 * 32 * 27)
    wd1 = torch.randn(9, 32, device="cuda")
    bd1 = torch.zeros(32, device="cuda")
    wp1 = torch.randn(16, 32, device="cuda") * 0.1
    bp1 = torch.zeros(16, device="cuda")
    us1 = timeit(lambda: torch.ops.nnsx.stem_ir1(xu, ws, bs, wd1, bd1, wp1, bp1, LUT))
    row("stem+block1 fused (replaces both)", us1,
        2 * B * 112 * 112 * (32 * 27 + 32 * 9 + 32 * 16))
    print(f"  fused saves {us + seen[(112, 32, 32, 16, 1)] - us1:.1f} us")
    xh = torch.randn(B * 49, 320, device="cuda")
    wh = torch.randn(1280, 320, device="cuda") * 0.05
    bh = torch.zeros(1280, device="cuda")
    us = timeit(lambda: torch.ops.nnsx.pw_conv(xh, wh, bh, None, 1280, 1, True))
    total += us
    row("head 320 -> 1280 (7x7)", us, 2 * B * 49 * 320 * 1280)
    xp = torch.randn(B, 7, 7, 1280, device="cuda")
    us = timeit(lambda: torch.ops.nnsx.avgpool(xp))
    total += us
    row("avgpool", us, B * 49 * 1280)
    xf = torch.randn(B, 1280, device="cuda")
    wf = torch.randn(1008, 1280, device="cuda") * 0.03
    bf = torch.zeros(1008, device="cuda")
    us = timeit(lambda: torch.ops.nnsx.pw_conv(xf, wf, bf, None, 1000, 0, True))
    total += us
    row("classifier 1280 -> 1000", us, 2 * B * 1280 * 1000)
    print(f"TOTAL {total:.1f} us per batch of {B}  ({B / total * 1e6:.0f} frames/s model-only)")
