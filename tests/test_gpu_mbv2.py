"""CDNA4 MobileNetV2 kernels (torch.ops.nnsx.*) vs PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _pw_ref(x, wt, bias, res, n, act, out_f32):
    k = x.shape[-1]
    v = x.float() @ wt[:n, :k].float().t() + bias[:n]
    if res is not None:
        v = v + res.float()
    if act == 1:
        v = v.clamp(0, 6)
    return v


@pytest.mark.parametrize("M,K,N", [(1000, 16, 96), (777, 24, 144), (4096, 144, 24), (3136, 320, 1280),
                                   (5, 1280, 1000), (130, 960, 160), (64, 32, 16)])
@pytest.mark.parametrize("act,use_res", [(1, False), (0, True)])
def test_pw_conv(nns, M, K, N, act, use_res):
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    npad, kpad = (N + 63) // 64 * 64, (K + 31) // 32 * 32
    wt = torch.zeros(npad, kpad, device="cuda")
    wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
    wt = wt.to(torch.bfloat16)
    bias = torch.randn(npad, device="cuda")
    res = torch.randn(M, N, device="cuda").to(torch.bfloat16) if use_res else None
    y = torch.ops.nnsx.pw_conv(x, wt, bias, res, N, act, False)
    ref = _pw_ref(x, wt, bias, res, N, act, False)
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)
    y32 = torch.ops.nnsx.pw_conv(x, wt, bias, res, N, act, True)
    torch.testing.assert_close(y32, ref, rtol=1e-3, atol=1e-3)


def test_pw_conv_identity_asymmetric(nns):
    # A = I check with asymmetric B catches transposed C/D layouts
    M, K, N = 64, 64, 64
    x = torch.arange(M * K, device="cuda", dtype=torch.float32).view(M, K).remainder(7).to(torch.bfloat16)
    wt = torch.eye(64, device="cuda").to(torch.bfloat16)
    y = torch.ops.nnsx.pw_conv(x, wt, torch.zeros(64, device="cuda"), None, N, 0, True)
    torch.testing.assert_close(y, x.float())


@pytest.mark.parametrize("B,H,W,C,stride", [(2, 112, 112, 32, 1), (3, 112, 112, 96, 2), (1, 7, 7, 960, 1),
                                            (2, 15, 9, 144, 2)])
def test_dw_conv(nns, B, H, W, C, stride):
    x = torch.randn(B, H, W, C, device="cuda").to(torch.bfloat16)
    w = torch.randn(9, C, device="cuda").to(torch.bfloat16)
    bias = torch.randn(C, device="cuda")
    y = torch.ops.nnsx.dw_conv(x, w, bias, stride, 1)
    wf = w.float().view(3, 3, C).permute(2, 0, 1).unsqueeze(1)
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), wf, bias, stride=stride, padding=1, groups=C).clamp(0, 6)
    torch.testing.assert_close(y.float(), ref.permute(0, 2, 3, 1), rtol=2e-2, atol=3e-2)


def test_stem_and_pool(nns):
    x = torch.randn(2, 224, 224, 3, device="cuda")
    w = torch.randn(3, 3, 3, 32, device="cuda") * 0.3
    b = torch.randn(32, device="cuda")
    y = torch.ops.nnsx.stem_conv(x, w, b, 1)
    ref = F.conv2d(x.permute(0, 3, 1, 2), w.permute(3, 2, 0, 1), b, stride=2, padding=1).clamp(0, 6)
    torch.testing.assert_close(y.float(), ref.permute(0, 2, 3, 1), rtol=2e-2, atol=3e-2)
    p = torch.ops.nnsx.avgpool(y)
    torch.testing.assert_close(p.float(), y.float().mean((1, 2)), rtol=2e-2, atol=2e-2)


def test_fused_mobilenet_matches_fp32_model(nns):
    from nnstreamer_amd.models.fused import FusedMobileNetV2
    from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2

    m = mobilenet_v2(seed=1).cuda()
    f = FusedMobileNetV2.from_reference(mobilenet_v2(seed=1)).cuda().eval()
    x = torch.rand(8, 224, 224, 3, device="cuda") * 2 - 1
    with torch.no_grad():
        ref = m(x.permute(0, 3, 1, 2))
        out = f(x)
        out_script = torch.jit.script(f)(x)
    err = (out - ref).abs().max().item()
    assert err < 0.05 * ref.abs().max().item(), err
    agree = (out.argmax(1) == ref.argmax(1)).float().mean().item()
    assert agree >= 0.75
    torch.testing.assert_close(out, out_script)
