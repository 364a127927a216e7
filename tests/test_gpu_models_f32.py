"""The fp32 (reference-precision) fused forms of the other BASELINE.json model
families on the GPU -- SSDLite-MobileNetV2 (config 3; heads writing straight
into the concatenated box / class tensors), DeepLabV3 (config 4), PoseNet
(config 5) -- against their plain fp32 PyTorch definitions on the same input.
The reference runs every model in float32 (tensor_filter_pytorch.cc:517-536)."""
import pytest
import torch

import nnstreamer_amd  # noqa: F401
from nnstreamer_amd.models import deeplab, posenet, ssd

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.float().flatten(), b.float().flatten()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _u8(b, s, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (b, s, s, 3), dtype=torch.uint8, generator=g).cuda()


def test_ssd_fp32_fused_matches_torch_fp32():
    m = ssd.ssd_mobilenet(seed=1).cuda().eval()
    f = torch.jit.script(ssd.FusedSSDLite.from_reference(ssd.ssd_mobilenet(seed=1), "fp32").cuda().eval())
    x = _u8(4, 300, 0)
    with torch.no_grad():
        fb, fc = f(x)
        b, c = m((x.float() - 127.5) / 127.5)
    assert fb.shape == (4, 1917, 1, 4) and fc.shape == (4, 1917, 91)
    assert _rel(fb, b) < 1e-3 and _rel(fc, c) < 1e-3, (_rel(fb, b), _rel(fc, c))


def test_deeplab_fp32_fused_matches_torch_fp32():
    m = deeplab.deeplabv3(seed=2).cuda().eval()
    f = torch.jit.script(deeplab.FusedDeepLabV3.from_reference(deeplab.deeplabv3(seed=2), "fp32").cuda().eval())
    x = _u8(2, 513, 1)
    with torch.no_grad():
        fy = f(x)
        y = m(x.float() / 255.0)
    assert fy.shape == y.shape == (2, 513, 513, 21)
    assert _rel(fy, y) < 1e-3, _rel(fy, y)
    # the segment decoder's decision: per-pixel argmax
    agree = (fy.argmax(-1) == y.argmax(-1)).float().mean().item()
    assert agree > 0.995, agree


def test_deeplab_fp32_lowres_and_kernels():
    """the lowres export (33x33 logits; the decoder resizes) and the hand-written
    NHWC bilinear resize / per-image-bias GEMM against their torch forms"""
    m = deeplab.deeplabv3(seed=2)
    f = torch.jit.script(deeplab.FusedDeepLabV3.from_reference(m, "fp32").cuda().eval())
    lo = torch.jit.script(deeplab.FusedDeepLabV3.from_reference(m, "fp32", lowres=True).cuda().eval())
    x = _u8(2, 513, 4)
    with torch.no_grad():
        fy = f(x)
        ly = lo(x)
    assert ly.shape == (2, 33, 33, 21)
    up = torch.ops.nnsx.upsample_bilinear(ly, 513, 513)
    assert torch.equal(up, fy)
    ref = torch.nn.functional.interpolate(ly.permute(0, 3, 1, 2), size=(513, 513), mode="bilinear",
                                          align_corners=True).permute(0, 2, 3, 1)
    assert _rel(up, ref) < 1e-6
    a = torch.randn(3, 33, 33, 256, device="cuda")
    wt = torch.randn(256, 256, device="cuda")
    bias = torch.randn(3, 256, device="cuda")
    r = torch.ops.nnsx.pw_conv_rowbias(a, wt, bias, 256, 1)
    exp = (a.double() @ wt.double().t() + bias.double().view(3, 1, 1, 256)).clamp(0, 6)
    assert _rel(r, exp) < 1e-5


def test_posenet_fp32_fused_matches_torch_fp32():
    m = posenet.posenet(seed=3).cuda().eval()
    f = torch.jit.script(posenet.FusedPoseNet.from_reference(posenet.posenet(seed=3), "fp32").cuda().eval())
    x = _u8(4, 257, 2)
    with torch.no_grad():
        fh, fo = f(x)
        h, o = m((x.float() - 127.5) / 127.5)
    assert _rel(fh, h) < 1e-3 and _rel(fo, o) < 1e-3, (_rel(fh, h), _rel(fo, o))


@pytest.mark.parametrize("H,cin,hid,cout,stride,dil", [
    (65, 32, 192, 32, 1, 1),     # odd maps: masked partial tiles
    (129, 24, 144, 24, 1, 1),
    (257, 16, 96, 24, 2, 1),
    (19, 64, 384, 64, 1, 1),     # SSD 19x19
])
def test_ir_block_dilated_and_partial_tiles(H, cin, hid, cout, stride, dil):
    """the fused inverted-residual kernel on map sizes no tile divides (DeepLab's
    257 / 129 / 65 / 33, SSD's 19), against the same op's host implementation"""
    g = torch.Generator().manual_seed(H + cin)
    B = 2
    kin = (cin + 7) // 8 * 8
    x = torch.rand(B, H, H, cin, generator=g)
    we = torch.randn(hid, kin, generator=g) * (2.0 / cin) ** 0.5
    be = torch.randn(hid, generator=g) * 0.1
    wd = torch.randn(9, hid, generator=g) * 0.3
    bd = torch.randn(hid, generator=g) * 0.1
    wp = torch.randn((cout + 15) // 16 * 16, hid, generator=g) * (1.0 / hid) ** 0.5
    bp = torch.randn(wp.shape[0], generator=g) * 0.1
    res = stride == 1 and cin == cout
    assert torch.ops.nnsx.ir_supported_f32(stride, H, H, cin, hid, cout, True, dil)
    args = (we, be, wd, bd, wp, bp)
    ref = torch.ops.nnsx.ir_block(x, *args, stride, cout, True, res, dil)
    got = torch.ops.nnsx.ir_block(x.cuda(), *[t.cuda() for t in args], stride, cout, True, res, dil).cpu()
    assert got.shape == ref.shape
    assert _rel(got, ref) < 1e-5, _rel(got, ref)


@pytest.mark.parametrize("B,HW,C", [(8, 33 * 33, 320), (512, 49, 1280), (3, 5, 12), (2, 1000, 36), (1, 300, 20)])
def test_avgpool_f32(B, HW, C):
    x = torch.randn(B, HW, 1, C, device="cuda")
    p = torch.ops.nnsx.avgpool(x)
    assert _rel(p.cpu(), x.double().cpu().mean((1, 2))) < 1e-6
    assert torch.equal(p, torch.ops.nnsx.avgpool(x))  # deterministic


@pytest.mark.parametrize("B", [1, 3, 64])
def test_sep_heads_one_launch_vs_fp64(B):
    """All 12 SSDLite heads (depthwise 3x3 + ReLU6 + predictor, box and class, 6
    maps) against an fp64 oracle of each head, rows of the concatenated outputs
    included: one grouped depthwise launch + one grouped GEMM launch
    (kernels/mbv2_f32.hip dw3x3_group / pw_gemm_group).  B = 64 is the benched
    batch (tiles spanning images at the 3x3 .. 1x1 maps)."""
    import torch.nn.functional as F

    m = ssd.fused_ssd_mobilenet(seed=3, precision="fp32").cuda()
    g = torch.Generator().manual_seed(5)
    shapes = [(19, 576), (10, 1280), (5, 512), (3, 256), (2, 256), (1, 128)]
    feats = [(torch.rand(B, s, s, c, generator=g) * 3).cuda() for s, c in shapes]
    rows = sum(s * s * (h.n // h.k) for (s, _), h in zip(shapes, m.box_heads))
    bo = torch.full((B, rows, 4), float("nan"), device="cuda")
    lo = torch.full((B, rows, 91), float("nan"), device="cuda")
    heads = list(m.cls_heads) + list(m.box_heads)
    torch.ops.nnsx.sep_heads(feats + feats, [h.dw.w for h in heads], [h.dw.bias for h in heads],
                             [h.pw.wt for h in heads], [h.pw.bias for h in heads], [h.n for h in heads],
                             [1] * 6 + [0] * 6, bo, lo, 0)

    def ref(x, h):
        C = x.shape[-1]
        wd = h.dw.w.double().cpu().t().reshape(C, 1, 3, 3)
        d = F.conv2d(x.double().cpu().permute(0, 3, 1, 2), wd, h.dw.bias.double().cpu(), padding=1,
                     groups=C).clamp(0, 6)
        w = h.pw.wt.double().cpu()[: h.n, :C]
        y = torch.einsum("bchw,nc->bhwn", d, w) + h.pw.bias.double().cpu()[: h.n]
        return y.reshape(x.shape[0], -1, h.k)

    for out, hs in ((lo, m.cls_heads), (bo, m.box_heads)):
        want = torch.cat([ref(x, h) for x, h in zip(feats, hs)], 1)
        got = out.double().cpu()
        assert not torch.isnan(got).any()
        err = ((got - want).abs() / (want.abs() + 1)).max().item()
        assert err < 2e-5, err


@pytest.mark.parametrize("shapes", [[(64, 17, 1024, 17, 0), (64, 17, 1024, 34, 0)],
                                    [(3, 7, 64, 13, 1), (2, 129, 32, 64, 1), (1, 1, 128, 4, 0)]])
def test_pw_conv_group_vs_fp64(shapes):
    """Several pointwise convs in one grouped GEMM launch (nnsx::pw_conv_group,
    kernels/mbv2_f32.hip pw_gemm_group_f32_kernel): exact-column NHWC outputs
    (the PoseNet heatmap + offset heads) against fp64."""
    g = torch.Generator().manual_seed(len(shapes))
    xs, wts, bs, ns, acts = [], [], [], [], []
    for B, H, K, N, act in shapes:
        xs.append((torch.rand(B, H, H, K, generator=g) * 2).cuda())
        w = torch.zeros((N + 7) // 8 * 8, K)
        w[:N] = torch.randn(N, K, generator=g) * K ** -0.5
        b = torch.zeros(w.shape[0])
        b[:N] = torch.randn(N, generator=g)
        wts.append(w.cuda())
        bs.append(b.cuda())
        ns.append(N)
        acts.append(act)
    outs = torch.ops.nnsx.pw_conv_group(xs, wts, bs, ns, acts)
    for x, w, b, n, act, y in zip(xs, wts, bs, ns, acts, outs):
        want = x.double().cpu() @ w.double().cpu()[:n].t() + b.double().cpu()[:n]
        if act:
            want = want.clamp(0, 6)
        assert y.shape == x.shape[:3] + (n,)
        err = ((y.double().cpu() - want).abs() / (want.abs() + 1)).max().item()
        assert err < 2e-5, err
