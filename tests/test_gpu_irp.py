"""The 14 x 14 image-per-workgroup inverted residual on split-bf16 MFMAs
(csrc/kernels/irp_x3.hip): the default kernel of MobileNetV2's 14 x 14 stage
under the x3 method.

Gate: against an fp64 oracle its max AND mean error are no
worse than the native fp32 MFMA kernel's on the same data -- no slack -- for
every shape it serves at the batches it serves (>= irp_min_batch, 128 by
default: below that the wave-split kernels keep the latency path), residual
and non-residual forms; bitwise repeatable.  Forced onto batches 1 and 3 (not a
default) its mean error stays below native's and its max within 10 % (one
image's 12.5k outputs make the max a single-sample statistic there: x3's mean
is ~35 % below native's, profiles/r6_x3_error_table.txt).  The reference
runs the block in float32 (tensor_filter_pytorch.cc:517-557)."""
import pytest
import torch

from test_gpu_mbv2_f32 import _ir_ref64
from test_gpu_x3 import _errs, _ir_weights

pytestmark = pytest.mark.gpu

IRP_SHAPES = [(64, 384, 64), (64, 384, 96), (96, 576, 96)]


@pytest.fixture
def method():
    prev = torch.ops.nnsx.f32_math()
    prev_b = torch.ops.nnsx.irp_min_batch(1)  # (small test batches take the kernel too)
    prev_h = torch.ops.nnsx.irh_mode(2)  # (the 28 x 28 half-image kernels: off by default)
    yield lambda m: torch.ops.nnsx.set_f32_math(m)
    torch.ops.nnsx.set_f32_math(prev)
    torch.ops.nnsx.irp_min_batch(prev_b)
    torch.ops.nnsx.irh_mode(prev_h)


@pytest.mark.parametrize("cin,hid,cout", IRP_SHAPES)
@pytest.mark.parametrize("B", [1, 3, 128, 512])
@pytest.mark.parametrize("dist", ["normal", "relu6"])
def test_irp_no_worse_than_native(nns, method, cin, hid, cout, B, dist):
    we, be, wd, bd, wp, bp, we3, wp3 = _ir_weights(cin, hid, cout, cin + hid + cout + B)
    x = torch.randn(B, 14, 14, cin, device="cuda")
    if dist == "relu6":  # what the previous block's project + residual feeds in MobileNetV2
        x = x * 2
    res = cin == cout
    ref = _ir_ref64(x, we, be, wd, bd, wp, bp, 1, cout, True, res)

    def run():
        return torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, 1, cout, True, res, 1, None, we3, wp3)

    method("fp32")
    y_nat = run()
    method("x3")
    assert torch.ops.nnsx.ir_method_f32(1, 14, 14, cin, hid, cout, B, 1) == "x3"
    y = run()
    assert not torch.equal(y, y_nat), "the x3 kernel did not run"
    (nat_max, nat_mean), (x3_max, x3_mean) = _errs(y_nat, ref), _errs(y, ref)
    slack = 1.0 if B >= 128 else 1.1  # (B < 128 is not served by default)
    assert x3_max <= nat_max * slack and x3_mean <= nat_mean, (nat_max, x3_max, nat_mean, x3_mean)
    assert torch.equal(y, run())


def test_irp_matches_wave_split_kernel(nns, method, monkeypatch):
    """same block through the previous default (irw, NNSX_IRP=0 in a child) and
    the new kernel: both within fp32 rounding of each other"""
    import os
    import subprocess
    import sys

    code = ("import torch, nnstreamer_amd, sys; sys.path.insert(0, 'tests');"
            "from test_gpu_x3 import _ir_weights;"
            "torch.ops.nnsx.irp_min_batch(1);"
            "w = _ir_weights(64, 384, 64, 5); torch.manual_seed(9); x = torch.randn(4, 14, 14, 64, device='cuda');"
            "y = torch.ops.nnsx.ir_block(x, *w[:6], 1, 64, True, True, 1, None, w[6], w[7]);"
            "torch.save(y.cpu(), sys.argv[1])")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    outs = []
    for flag in ("0", "1"):
        path = f"/tmp/irp_ab_{os.getpid()}_{flag}.pt"
        env = dict(os.environ, NNSX_IRP=flag)
        r = subprocess.run([sys.executable, "-c", code, path], cwd=root, env=env, capture_output=True, text=True,
                           timeout=300)
        assert r.returncode == 0, r.stderr[-2000:]
        outs.append(torch.load(path, weights_only=True))
        os.unlink(path)
    assert not torch.equal(outs[0], outs[1])
    assert (outs[0] - outs[1]).abs().max().item() < 1e-4


@pytest.mark.parametrize("H,cin,hid,cout,stride", [(14, 96, 576, 160, 2), (28, 32, 192, 32, 1),
                                                    (28, 32, 192, 64, 2)])
@pytest.mark.parametrize("B", [1, 3, 128, 512])
@pytest.mark.parametrize("dist", ["normal", "relu6"])
def test_irp_other_maps_no_worse_than_native(nns, method, H, cin, hid, cout, stride, B, dist):
    """the stride-2 14 x 14 -> 7 x 7 block (96 -> 576 -> 160, irps_x3_kernel) and
    the 28 x 28 32 -> 192 -> 32 and 28 -> 14 32 -> 192 -> 64 blocks (half an
    image per workgroup, irh_x3_kernel): same gate as the 14 x 14 stride-1
    shapes"""
    we, be, wd, bd, wp, bp, we3, wp3 = _ir_weights(cin, hid, cout, 7 + B + H)
    x = torch.randn(B, H, H, cin, device="cuda")
    if dist == "relu6":
        x = (x * 2).clamp(0, 6)
    res = stride == 1 and cin == cout
    ref = _ir_ref64(x, we, be, wd, bd, wp, bp, stride, cout, True, res)

    def run():
        return torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res, 1, None, we3, wp3)

    method("fp32")
    y_nat = run()
    method("x3")
    assert torch.ops.nnsx.ir_method_f32(stride, H, H, cin, hid, cout, B, 1) == "x3"
    y = run()
    Ho = (H - 1) // stride + 1
    assert y.shape == (B, Ho, Ho, cout)
    assert not torch.equal(y, y_nat), "the x3 kernel did not run"
    (nat_max, nat_mean), (x3_max, x3_mean) = _errs(y_nat, ref), _errs(y, ref)
    slack = 1.0 if B >= 128 else 1.1
    assert x3_max <= nat_max * slack and x3_mean <= nat_mean, (nat_max, x3_max, nat_mean, x3_mean)
    assert torch.equal(y, run())
