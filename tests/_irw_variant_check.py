"""Child process of test_gpu_mbv2_f32.py::test_irw_tile_variants: the fused
fp32 inverted-residual kernel under NNSX_IRW_SKIP (read once at library load,
so the A/B tile configurations need their own process) vs the fp64 oracle,
bitwise repeatable.  argv: H,cin,hid,cout,stride;... batch list"""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __file__.rsplit("/tests/", 1)[0])
import nnstreamer_amd  # noqa: F401,E402  (registers torch.ops.nnsx)


def ref64(x, we, be, wd, bd, wp, bp, stride, cout, residual):
    x64 = x.double().cpu()
    cin, hid = x.shape[-1], wd.shape[1]
    h = (x64 @ we.double().cpu()[:, :cin].t() + be.double().cpu()).clamp(0, 6)
    wdf = wd.double().cpu().view(3, 3, hid).permute(2, 0, 1).unsqueeze(1)
    h = F.conv2d(h.permute(0, 3, 1, 2), wdf, bd.double().cpu(), stride=stride, padding=1, groups=hid).clamp(0, 6)
    y = h.permute(0, 2, 3, 1) @ wp.double().cpu()[:cout].t() + bp.double().cpu()[:cout]
    return y + x64 if residual else y


def main():
    shapes = [tuple(int(v) for v in s.split(",")) for s in sys.argv[1].split(";")]
    batches = [int(b) for b in sys.argv[2].split(",")]
    worst = 0.0
    for H, cin, hid, cout, stride in shapes:
        for B in batches:
            torch.manual_seed(H + cin + hid + cout + B)
            x = torch.randn(B, H, H, cin, device="cuda")
            kin = (cin + 7) // 8 * 8
            we = torch.zeros(hid, kin, device="cuda")
            we[:, :cin] = torch.randn(hid, cin, device="cuda") / cin ** 0.5
            be = torch.randn(hid, device="cuda") * 0.1
            wd = torch.randn(9, hid, device="cuda") / 3
            bd = torch.randn(hid, device="cuda") * 0.1
            npad = (cout + 15) // 16 * 16
            wp = torch.zeros(npad, hid, device="cuda")
            wp[:cout] = torch.randn(cout, hid, device="cuda") / hid ** 0.5
            bp = torch.zeros(npad, device="cuda")
            bp[:cout] = torch.randn(cout, device="cuda") * 0.1
            res = stride == 1 and cin == cout
            y = torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res)
            y2 = torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res)
            assert torch.equal(y, y2), (H, cin, hid, cout, B)
            r = ref64(x, we, be, wd, bd, wp, bp, stride, cout, res)
            err = (y.double().cpu() - r).abs().max().item() / max(1.0, r.abs().max().item())
            assert err <= 5e-5, (H, cin, hid, cout, B, err)
            worst = max(worst, err)
    print(f"OK worst {worst:.3g}")


if __name__ == "__main__":
    main()
