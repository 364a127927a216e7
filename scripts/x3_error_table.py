"""Per-shape error table of the fp32 engine's two product methods -- native
v_mfma_f32 (`fp32`) and split-bf16 (`x3`) -- for every MobileNetV2 inverted
residual the x3 method serves by default, at the benched batch (VERDICT r5
item 6).  Errors against an fp64 oracle of the same block on the same data:
max and mean of |y - ref| / max(1, max |ref|); input drawn as the previous
block feeds it (relu6-range); `kernel` is what ir_method_f32 picks.

    python scripts/x3_error_table.py [--batch 512] [--seeds 2] [--only H,cin,hid,cout,s] [--dist relu6|normal]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402
from test_gpu_mbv2_f32 import _ir_ref64  # noqa: E402
from test_gpu_x3 import _errs, _ir_weights  # noqa: E402

# MobileNetV2 (width 1.0, 224) expanded blocks: (H_in, cin, hid, cout, stride)
BLOCKS = [
    (112, 16, 96, 24, 2), (56, 24, 144, 24, 1), (56, 24, 144, 32, 2), (28, 32, 192, 32, 1),
    (28, 32, 192, 64, 2), (14, 64, 384, 64, 1), (14, 64, 384, 96, 1), (14, 96, 576, 96, 1),
    (14, 96, 576, 160, 2), (7, 160, 960, 160, 1), (7, 160, 960, 320, 1),
]
# (14 -> 7 96 -> 576 -> 160 serves by default only where its gate passes; --only forces it)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--seeds", type=int, default=2)
    ap.add_argument("--only", default="", help="one block H,cin,hid,cout,stride")
    ap.add_argument("--dist", default="relu6", choices=["relu6", "normal"])
    a = ap.parse_args()
    blocks = [tuple(int(v) for v in a.only.split(","))] if a.only else BLOCKS
    prev = torch.ops.nnsx.f32_math()
    print(f"# x3 vs native fp32 error per default-x3 block, B={a.batch}, input {a.dist}, "
          f"{torch.cuda.get_device_name(0)}")
    print(f"{'block':28s} {'seed':>4s} {'kernel':>6s} | {'native max':>11s} {'x3 max':>11s} {'ratio':>6s} | "
          f"{'native mean':>11s} {'x3 mean':>11s} {'ratio':>6s}")
    worst = 0.0
    for H, cin, hid, cout, s in blocks:
        torch.ops.nnsx.set_f32_math("x3")
        m = torch.ops.nnsx.ir_method_f32(s, H, H, cin, hid, cout, a.batch, 1)
        if m != "x3":
            continue
        res = s == 1 and cin == cout
        for seed in range(a.seeds):
            we, be, wd, bd, wp, bp, we3, wp3 = _ir_weights(cin, hid, cout, 1000 * seed + cin + hid + cout)
            x = torch.randn(a.batch, H, H, cin, device="cuda")
            if a.dist == "relu6":
                x = (x * 2).clamp(0, 6)
            ref = _ir_ref64(x, we, be, wd, bd, wp, bp, s, cout, True, res)
            out = {}
            for meth in ("fp32", "x3"):
                torch.ops.nnsx.set_f32_math(meth)
                out[meth] = _errs(torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, s, cout, True, res, 1, None,
                                                          we3, wp3), ref)
            (nmax, nmean), (xmax, xmean) = out["fp32"], out["x3"]
            worst = max(worst, xmax / nmax)
            print(f"{H}x{H} {cin}->{hid}->{cout} s{s}".ljust(28) + f" {seed:4d} {'x3':>6s} | {nmax:11.3e} {xmax:11.3e} "
                  f"{xmax / nmax:6.3f} | {nmean:11.3e} {xmean:11.3e} {xmean / nmean:6.3f}", flush=True)
            del ref, x
    torch.ops.nnsx.set_f32_math(prev)
    print(f"# worst x3/native max-error ratio: {worst:.3f}")


if __name__ == "__main__":
    main()
