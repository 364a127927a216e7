"""fp32 CDNA4 MobileNetV2 kernels (csrc/kernels/mbv2_f32.hip) vs float64
references, plus model- and pipeline-level agreement gates for the benched
engines (fp32 = reference precision, bf16 = secondary)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from nnstreamer_amd.models.fused import input_lut

pytestmark = pytest.mark.gpu


def _close(y, ref, tol=2e-5):
    """fp32 kernel vs fp64 oracle: relative to the output's scale."""
    y = y.double().cpu()
    ref = ref.double().cpu()
    scale = max(1.0, ref.abs().max().item())
    err = (y - ref).abs().max().item()
    assert err <= tol * scale, f"max abs err {err} (scale {scale})"


@pytest.mark.parametrize("M,K,N", [(1000, 16, 96), (777, 24, 144), (4096, 144, 24), (6272, 320, 1280),
                                   (128, 1280, 1000), (130, 960, 160), (64, 32, 16), (6272, 160, 960),
                                   (6272, 960, 320), (8712, 960, 160)])
@pytest.mark.parametrize("act,use_res", [(1, False), (0, True), (0, False)])
def test_pw_conv_f32(nns, M, K, N, act, use_res):
    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device="cuda")
    npad, kpad = (N + 15) // 16 * 16, (K + 7) // 8 * 8
    wt = torch.zeros(npad, kpad, device="cuda")
    wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
    bias = torch.randn(npad, device="cuda")
    res = torch.randn(M, N, device="cuda") if use_res else None
    y = torch.ops.nnsx.pw_conv(x, wt, bias, res, N, act, True)
    assert y.dtype == torch.float32
    ref = x.double().cpu() @ wt[:N, :K].double().cpu().t() + bias[:N].double().cpu()
    if use_res:
        ref = ref + res.double().cpu()
    if act == 1:
        ref = ref.clamp(0, 6)
    _close(y, ref)


def test_pw_conv_f32_identity_asymmetric(nns):
    # A = I with an asymmetric B catches transposed fragment / k-permutation bugs exactly
    M, K, N = 192, 64, 64
    x = torch.arange(M * K, device="cuda", dtype=torch.float32).view(M, K).remainder(13) - 6
    wt = torch.eye(64, device="cuda")
    y = torch.ops.nnsx.pw_conv(x, wt, torch.zeros(64, device="cuda"), None, N, 0, True)
    torch.testing.assert_close(y, x, rtol=0, atol=0)


@pytest.mark.parametrize("B,H,W,C,stride,dil", [(2, 112, 112, 32, 1, 1), (3, 112, 112, 96, 2, 1), (1, 7, 7, 960, 1, 1),
                                                (2, 15, 9, 144, 2, 1), (2, 33, 33, 320, 1, 2), (1, 65, 65, 64, 1, 4),
                                                # partial row / column groups of the 4 x 4 (stride 1) and
                                                # 2 x 2 (stride 2) lanes; SSD's tiny extras
                                                (2, 13, 11, 64, 1, 1), (1, 5, 6, 16, 2, 1), (3, 17, 17, 512, 1, 1),
                                                (2, 129, 129, 64, 2, 1), (1, 1, 1, 128, 1, 1), (2, 2, 2, 256, 2, 1),
                                                (1, 3, 3, 256, 2, 1), (1, 17, 13, 64, 1, 2), (3, 5, 5, 32, 1, 2),
                                                # (maps large enough for the multi-pixel lanes, partial groups)
                                                (8, 45, 43, 256, 1, 1), (16, 33, 33, 288, 1, 2),
                                                (8, 129, 129, 64, 2, 1),
                                                # dilation 2 residue-grid lanes (4 x 4 large, 2 x 2 small;
                                                # even / odd extents)
                                                (8, 33, 33, 960, 1, 2), (16, 34, 31, 256, 1, 2),
                                                (1, 33, 33, 960, 1, 2), (2, 34, 31, 64, 1, 2)])
@pytest.mark.parametrize("act", [1, 3])
def test_dw_conv_f32(nns, B, H, W, C, stride, dil, act):
    """act 3 = the producer's deferred ReLU6 applied to the input taps, then ReLU6"""
    x = torch.randn(B, H, W, C, device="cuda") * 4
    w = torch.randn(9, C, device="cuda")
    bias = torch.randn(C, device="cuda")
    y = torch.ops.nnsx.dw_conv(x, w, bias, stride, act, dil)
    assert y.dtype == torch.float32
    wf = w.double().cpu().view(3, 3, C).permute(2, 0, 1).unsqueeze(1)
    xin = x.double().cpu().permute(0, 3, 1, 2)
    if act == 3:
        xin = xin.clamp(0, 6)
    ref = F.conv2d(xin, wf, bias.double().cpu(), stride=stride, padding=dil, dilation=dil, groups=C).clamp(0, 6)
    _close(y, ref.permute(0, 2, 3, 1))


@pytest.mark.parametrize("H,W", [(224, 224), (300, 300), (57, 41)])
def test_stem_f32_u8_and_pool(nns, H, W):
    x = torch.randint(0, 256, (2, H, W, 3), device="cuda", dtype=torch.uint8)
    w = torch.randn(3, 3, 3, 32, device="cuda") * 0.3
    b = torch.randn(32, device="cuda")
    y = torch.ops.nnsx.stem_conv_u8(x, w, b, 1, input_lut(-127.5, 127.5).cuda(), True)
    assert y.dtype == torch.float32
    xf = (x.double().cpu() - 127.5) / 127.5
    ref = F.conv2d(xf.permute(0, 3, 1, 2), w.double().cpu().permute(3, 2, 0, 1), b.double().cpu(), stride=2,
                   padding=1).clamp(0, 6)
    _close(y, ref.permute(0, 2, 3, 1))
    yf = torch.ops.nnsx.stem_conv(((x.float() - 127.5) / 127.5).contiguous(), w, b, 1, True)
    _close(yf, ref.permute(0, 2, 3, 1))
    p = torch.ops.nnsx.avgpool(y)
    _close(p, y.double().cpu().mean((1, 2)))


@pytest.mark.parametrize("H,W,B", [(224, 224, 3), (300, 300, 2), (57, 41, 2), (17, 35, 1), (513, 513, 1),
                                   (224, 224, 20)])
def test_stem_ir1_f32(nns, H, W, B):
    """stem + first block fused (uint8 frame -> 16 channels, one wave per 8 x 8
    tile) vs the fp64 chain"""
    torch.manual_seed(H + W)
    x = torch.randint(0, 256, (B, H, W, 3), device="cuda", dtype=torch.uint8)
    ws = torch.randn(3, 3, 3, 32, device="cuda") * 0.3
    bs = torch.randn(32, device="cuda") * 0.1
    wd = torch.randn(9, 32, device="cuda") / 3
    bd = torch.randn(32, device="cuda") * 0.1
    wp = torch.randn(16, 32, device="cuda") / 32 ** 0.5
    bp = torch.randn(16, device="cuda") * 0.1
    y = torch.ops.nnsx.stem_ir1(x, ws, bs, wd, bd, wp, bp, input_lut(-127.5, 127.5).cuda())
    assert y.shape == (B, (H - 1) // 2 + 1, (W - 1) // 2 + 1, 16) and y.dtype == torch.float32
    xf = (x.double().cpu() - 127.5) / 127.5
    h = F.conv2d(xf.permute(0, 3, 1, 2), ws.double().cpu().permute(3, 2, 0, 1), bs.double().cpu(), stride=2,
                 padding=1).clamp(0, 6)
    h = F.conv2d(h, wd.double().cpu().view(3, 3, 32).permute(2, 0, 1).unsqueeze(1), bd.double().cpu(), padding=1,
                 groups=32).clamp(0, 6)
    ref = h.permute(0, 2, 3, 1) @ wp.double().cpu().t() + bp.double().cpu()
    _close(y, ref, tol=5e-5)


# every fused MobileNetV2 block (H, cin, hid, cout, stride, expand) + partial-tile shapes
IR_F32_SHAPES = [(112, 32, 32, 16, 1, False), (112, 16, 96, 24, 2, True), (56, 24, 144, 24, 1, True),
                 (56, 24, 144, 32, 2, True), (28, 32, 192, 32, 1, True), (28, 32, 192, 64, 2, True),
                 (14, 64, 384, 64, 1, True), (14, 64, 384, 96, 1, True), (14, 96, 576, 96, 1, True),
                 (21, 64, 384, 64, 1, True), (13, 96, 576, 96, 1, True), (15, 32, 192, 64, 2, True),
                 (42, 32, 192, 32, 1, True), (40, 16, 96, 24, 2, True),
                 (30, 24, 144, 24, 1, True), (17, 64, 384, 96, 1, True),
                 # wave-split kernel: 7x7 whole-image tiles with the hidden channels split over 2 workgroups
                 (7, 160, 960, 160, 1, True), (35, 96, 576, 96, 1, True),
                 # 14 -> 7 stride-2 block (B14): one 7x7 image per tile, 3 waves
                 (14, 96, 576, 160, 2, True),
                 # SSD-300's 10x10 stage on exact 5x5 tiles
                 (10, 160, 960, 160, 1, True), (19, 96, 576, 160, 2, True),
                 # SSD-300's 19x19 stage on masked 5x5 tiles (the least-padding pick)
                 (19, 64, 384, 64, 1, True), (19, 64, 384, 96, 1, True), (19, 96, 576, 96, 1, True),
                 # DeepLab's 33x33, 65x65 and 129x129 maps, SSD's 38x38 and 75x75 (5 x 10 / 5 x 15 tiles)
                 (33, 64, 384, 64, 1, True), (33, 96, 576, 96, 1, True), (65, 32, 192, 32, 1, True),
                 (38, 32, 192, 32, 1, True), (75, 24, 144, 24, 1, True), (129, 24, 144, 24, 1, True)]


def _ir_ref64(x, we, be, wd, bd, wp, bp, stride, cout, has_expand, residual, dil=1):
    x64 = x.double().cpu()
    cin = x.shape[-1]
    hid = wd.shape[1]
    h = x64
    if has_expand:
        h = (x64 @ we.double().cpu()[:, :cin].t() + be.double().cpu()).clamp(0, 6)
    wdf = wd.double().cpu().view(3, 3, hid).permute(2, 0, 1).unsqueeze(1)
    h = F.conv2d(h.permute(0, 3, 1, 2), wdf, bd.double().cpu(), stride=stride, padding=dil, dilation=dil,
                 groups=hid).clamp(0, 6)
    h = h.permute(0, 2, 3, 1)
    y = h @ wp.double().cpu()[:cout].t() + bp.double().cpu()[:cout]
    if residual:
        y = y + x64
    return y


@pytest.mark.parametrize("H,cin,hid,cout,stride,has_expand", IR_F32_SHAPES)
@pytest.mark.parametrize("B", [3, 1])
def test_ir_block_f32(nns, H, cin, hid, cout, stride, has_expand, B):
    torch.manual_seed(H * 7 + cin + hid)
    assert torch.ops.nnsx.ir_supported_f32(stride, H, H, cin, hid, cout, has_expand)
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
    residual = stride == 1 and cin == cout
    y = torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, has_expand, residual)
    assert y.shape == (B, (H - 1) // stride + 1, (H - 1) // stride + 1, cout)
    _close(y, _ir_ref64(x, we, be, wd, bd, wp, bp, stride, cout, has_expand, residual), tol=5e-5)


@pytest.mark.parametrize("H,cin,hid,cout,stride", [(7, 160, 960, 160, 1), (14, 96, 576, 160, 2)])
def test_ir_block_f32_two_parts_deterministic(nns, H, cin, hid, cout, stride):
    """batch 128 on the 7x7 blocks: 128 tiles -> two hidden parts per tile
    (workspace slabs + ordered reduce); bitwise repeatable."""
    torch.manual_seed(cin + hid)
    B = 128
    x = torch.randn(B, H, H, cin, device="cuda")
    we = torch.randn(hid, cin, device="cuda") / cin ** 0.5
    be = torch.randn(hid, device="cuda") * 0.1
    wd = torch.randn(9, hid, device="cuda") / 3
    bd = torch.randn(hid, device="cuda") * 0.1
    wp = torch.randn(cout, hid, device="cuda") / hid ** 0.5
    bp = torch.randn(cout, device="cuda") * 0.1
    res = stride == 1 and cin == cout
    y = torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res)
    y2 = torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res)
    assert torch.equal(y, y2)
    _close(y, _ir_ref64(x, we, be, wd, bd, wp, bp, stride, cout, True, res), tol=5e-5)


@pytest.mark.parametrize("H,cin,hid,cout,stride", [(56, 24, 144, 24, 1), (28, 32, 192, 64, 2), (14, 64, 384, 96, 1),
                                                    (14, 96, 576, 160, 2), (7, 160, 960, 160, 1),
                                                    (33, 64, 384, 64, 1)])
@pytest.mark.parametrize("B", [1, 2, 8])
def test_ir_block_f32_inlaunch_combine(nns, H, cin, hid, cout, stride, B):
    """Hidden parts combined inside the launch (the model's ticket buffer;
    NNSX_F32_IRW_INLAUNCH=1 last arriver, =2 every part adds its share after a
    per-tile arrival count) == the separate ordered reduce launch, bitwise, over
    repeated launches on one ticket buffer (monotone counters).  Batch 8 of the
    33x33 block (DeepLab: 200 tiles x 2 parts, more than the chip holds) takes
    the last-arriver form in its own ticket region."""
    torch.manual_seed(cin + hid + B)
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
    tickets = torch.zeros(768, dtype=torch.int32, device="cuda")
    ref = torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res, 1, None)
    for _ in range(3):
        y = torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res, 1, tickets)
        assert torch.equal(y, ref)
    _close(ref, _ir_ref64(x, we, be, wd, bd, wp, bp, stride, cout, True, res), tol=5e-5)


@pytest.mark.parametrize("skip", ["7,8,9", "6", "0,1,2,3,4"])
def test_irw_tile_variants(skip):
    """The A/B tile configurations of the fused block (7 x 14 tiles on the
    14 x 14 blocks; 8 x 8 / 8 x 16 / 4 x 8 / 7 x 14 tiles on the 112 / 56 / 28
    blocks), selected with NNSX_IRW_SKIP in a child process, vs fp64 and
    bitwise repeatable."""
    import os
    import subprocess
    import sys

    # (kIrwCfgs indices: 6 = the 7 x 14 64 -> 384 -> 64 default for batch >= 16,
    # 7-9 = the 7 x 7 14x14 configurations, 0-4 = the 112 / 56 / 28 defaults)
    shapes = ("14,64,384,64,1;14,64,384,96,1;14,96,576,96,1" if skip in ("7,8,9", "6")
              else "112,16,96,24,2;56,24,144,24,1;56,24,144,32,2;28,32,192,32,1")
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "_irw_variant_check.py"), shapes, "1,3,16,32"],
                       env=dict(os.environ, NNSX_IRW_SKIP=skip), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]


@pytest.mark.parametrize("B", [128, 3, 1])
def test_ir_expand_dw_f32(nns, B):
    """expand + depthwise in one kernel, depthwise output to HBM (the 7x7
    160 -> 960 block whose project to 320 runs as a GEMM) vs fp64."""
    torch.manual_seed(B)
    cin, hid, H = 160, 960, 7
    assert torch.ops.nnsx.ir_expand_dw_supported_f32(1, H, H, cin, hid)
    x = torch.randn(B, H, H, cin, device="cuda")
    we = torch.randn(hid, cin, device="cuda") / cin ** 0.5
    be = torch.randn(hid, device="cuda") * 0.1
    wd = torch.randn(9, hid, device="cuda") / 3
    bd = torch.randn(hid, device="cuda") * 0.1
    y = torch.ops.nnsx.ir_expand_dw(x, we, be, wd, bd, 1)
    h = (x.double().cpu() @ we.double().cpu().t() + be.double().cpu()).clamp(0, 6)
    ref = F.conv2d(h.permute(0, 3, 1, 2), wd.double().cpu().view(3, 3, hid).permute(2, 0, 1).unsqueeze(1),
                   bd.double().cpu(), padding=1, groups=hid).clamp(0, 6).permute(0, 2, 3, 1)
    _close(y, ref, tol=5e-5)


@pytest.mark.parametrize("M,K,N,act,use_res", [(1, 1280, 1000, 0, False), (5, 1280, 1000, 0, False),
                                                (17, 320, 1280, 1, False), (33, 960, 320, 0, True),
                                                (49, 960, 320, 0, False), (64, 96, 160, 1, True), (49, 36, 24, 0, False)])
def test_pw_small_m_f32(nns, M, K, N, act, use_res):
    """small-M GEMMs vs fp64, bitwise repeatable: M <= 16 or K <= 512 take the one-launch path (k-slices
    added through LDS in order), the deep-K many-row shapes (33 / 49 x 960) the split-K GEMM + reduce"""
    torch.manual_seed(M * K + N)
    x = torch.randn(M, K, device="cuda")
    kpad, npad = (K + 7) // 8 * 8, (N + 15) // 16 * 16
    wt = torch.zeros(npad, kpad, device="cuda")
    wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
    bias = torch.zeros(npad, device="cuda")
    bias[:N] = torch.randn(N, device="cuda") * 0.1
    res = torch.randn(M, N, device="cuda") if use_res else None
    y = torch.ops.nnsx.pw_conv(x, wt, bias, res, N, act, True)
    y2 = torch.ops.nnsx.pw_conv(x, wt, bias, res, N, act, True)
    assert torch.equal(y, y2)
    ref = x.double().cpu() @ wt.double().cpu()[:N, :K].t() + bias.double().cpu()[:N]
    if act == 1:
        ref = ref.clamp(0, 6)
    if use_res:
        ref = ref + res.double().cpu()
    _close(y, ref, tol=5e-5)


@pytest.mark.parametrize("B,H", [(1, 7), (3, 7), (2, 10)])
def test_pw_conv_pool_f32(nns, B, H):
    """head 1x1 conv + ReLU6 + global average pool in one launch vs fp64"""
    torch.manual_seed(B * 100 + H)
    K, N = 320, 1280
    x = torch.randn(B, H, H, K, device="cuda")
    wt = torch.randn(N, K, device="cuda") / K ** 0.5
    bias = torch.randn(N, device="cuda") * 0.1
    y = torch.ops.nnsx.pw_conv_pool(x, wt, bias, N, 1)
    assert y.shape == (B, N)
    ref = (x.double().cpu() @ wt.double().cpu().t() + bias.double().cpu()).clamp(0, 6).mean((1, 2))
    _close(y, ref, tol=5e-5)


@pytest.mark.parametrize("B,H", [(9, 7), (64, 7), (171, 7), (12, 8)])
def test_pw_conv_pool_f32_gemm_epilogue(nns, B, H):
    """larger batches: the tiled GEMM's pooling epilogue (64- and 128-row tiles,
    images straddling two row tiles: two order-free addends) vs fp64, bitwise
    repeatable, and equal within fp32 rounding to the head GEMM + avgpool pair"""
    torch.manual_seed(B * 7 + H)
    K, N = 320, 1280
    x = torch.randn(B, H, H, K, device="cuda")
    wt = torch.randn(N, K, device="cuda") / K ** 0.5
    bias = torch.randn(N, device="cuda") * 0.1
    ys = [torch.ops.nnsx.pw_conv_pool(x, wt, bias, N, 1) for _ in range(3)]
    assert all(torch.equal(ys[0], y) for y in ys[1:])
    ref = (x.double().cpu() @ wt.double().cpu().t() + bias.double().cpu()).clamp(0, 6).mean((1, 2))
    _close(ys[0], ref, tol=5e-5)
    two = torch.ops.nnsx.avgpool(torch.ops.nnsx.pw_conv(x, wt, bias, None, N, 1, True))
    assert (ys[0] - two).abs().max().item() < 1e-5


def test_classifier_split_k_deterministic(nns):
    """M = batch GEMM (split over K, slabs added in order): bitwise repeatable."""
    torch.manual_seed(5)
    x = torch.randn(128, 1280, device="cuda")
    wt = torch.randn(1008, 1280, device="cuda") / 1280 ** 0.5
    bias = torch.randn(1008, device="cuda")
    ys = [torch.ops.nnsx.pw_conv(x, wt, bias, None, 1000, 0, True) for _ in range(3)]
    assert all(torch.equal(ys[0], y) for y in ys[1:])
    _close(ys[0], x.double().cpu() @ wt[:1000].double().cpu().t() + bias[:1000].double().cpu())


def _agreement(f, m, n_images=256, batch=64, seed=0):
    g = torch.Generator().manual_seed(seed)
    agree, worst = 0, 0.0
    for _ in range(n_images // batch):
        x = torch.randint(0, 256, (batch, 224, 224, 3), generator=g, dtype=torch.uint8).cuda()
        with torch.no_grad():
            ref = m(((x.float() - 127.5) / 127.5).permute(0, 3, 1, 2))
            out = f(x)
        agree += int((out.argmax(1) == ref.argmax(1)).sum())
        worst = max(worst, ((out - ref).abs().max() / ref.abs().max()).item())
    return agree / n_images, worst


def test_fused_fp32_mobilenet_top1_matches_torch_fp32(nns):
    """The benched headline engine: fp32 fused kernels vs the plain torch fp32
    model on 256 images -- top-1 agreement >= 99.5 %."""
    from nnstreamer_amd.models.fused import FusedMobileNetV2
    from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2

    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    m = mobilenet_v2(seed=1).cuda().eval()
    f = torch.jit.script(FusedMobileNetV2.from_reference(mobilenet_v2(seed=1), "fp32").cuda().eval())
    agree, worst = _agreement(f, m)
    assert agree >= 0.995, (agree, worst)
    assert worst < 1e-3, worst


def test_fused_fp32_mobilenet_bench_batch_matches_torch_fp32(nns):
    """The same gate at bench.py's batch (512 frames per invoke: every block
    runs one hidden part per tile, the persistent stem walks 2 tiles per
    workgroup more than at 128)."""
    from nnstreamer_amd.models.fused import FusedMobileNetV2
    from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2

    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    m = mobilenet_v2(seed=2).cuda().eval()
    f = torch.jit.script(FusedMobileNetV2.from_reference(mobilenet_v2(seed=2), "fp32").cuda().eval())
    agree, worst = _agreement(f, m, n_images=512, batch=512, seed=2)
    assert agree >= 0.995, (agree, worst)
    assert worst < 1e-3, worst


def test_fused_bf16_mobilenet_top1_matches_torch_fp32(nns):
    """The secondary bf16 engine: top-1 agreement with torch fp32 >= 98 %."""
    from nnstreamer_amd.models.fused import FusedMobileNetV2
    from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2

    m = mobilenet_v2(seed=1).cuda().eval()
    f = torch.jit.script(FusedMobileNetV2.from_reference(mobilenet_v2(seed=1), "bf16").cuda().eval())
    agree, worst = _agreement(f, m)
    assert agree >= 0.98, (agree, worst)


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_benched_launch_string_labels_match_torch_fp32(nns, workdir, labels, precision):
    """The exact bench.py pipeline shape (uint8 frames -> stem-normalised fused
    model under hipGraph -> image_labeling) against torch.argmax of the plain
    fp32 model on the same frames."""
    import os

    from nnstreamer_amd.models.export import export
    from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2

    name = "mobilenet_v2_fused_fp32" if precision == "fp32" else "mobilenet_v2_fused"
    model = export(name, os.path.join(workdir, f"{name}.pt"), layout="nhwc")
    B, nb = 16, 4
    desc = (f"videotestsrc num-buffers={B * nb} pattern=snow pool-size=64 "
            "! video/x-raw,format=RGB,width=224,height=224,framerate=0/1 "
            f"! tee name=t t. ! queue ! tensor_converter frames-per-tensor={B} device=0 ! queue max-size-buffers=2 "
            f"! tensor_filter framework=pytorch model={model} input=3:224:224:{B} inputtype=uint8 "
            "accelerator=true:gpu device=0 custom=hipgraph:true ! queue max-size-buffers=4 "
            f"! tensor_decoder mode=image_labeling option1={labels} ! tensor_sink name=sink "
            f"t. ! queue ! tensor_converter frames-per-tensor={B} ! appsink name=raw")
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes().decode()))
    raw = p.get_by_name("raw")
    p.set_state("playing")
    frames = []
    while len(frames) < nb:
        b = raw.pull(timeout=60)
        assert b is not None
        frames.append(b.memory(0).numpy("uint8").copy())
    p.wait(timeout=120)
    p.stop()
    assert len(out) == nb
    m = mobilenet_v2(seed=0).cuda().eval()  # export() uses seed 0
    agree = total = 0
    for labels_txt, fr in zip(out, frames):
        x = torch.from_numpy(fr).cuda().view(B, 224, 224, 3).float()
        with torch.no_grad():
            ref = m(((x - 127.5) / 127.5).permute(0, 3, 1, 2)).argmax(1).tolist()
        got = labels_txt.split("\n")
        agree += sum(a == f"class_{i}" for a, i in zip(got, ref))
        total += B
    need = 1.0 if precision == "fp32" else 0.95
    assert agree / total >= need, (agree, total)


def test_replay_lanes_same_labels(nns, workdir, labels):
    """custom=lanes:<n>: consecutive batches replay round robin on n streams
    (own graphs and memory pool per lane; the in-launch combine then never
    waits on other workgroups).  Every frame's label equals the one-lane run,
    in order, with the absorbed argmax's indices read back on the lanes."""
    import os

    from nnstreamer_amd.models.export import export

    model = export("mobilenet_v2_fused_fp32", os.path.join(workdir, "mbv2_f32_lanes.pt"), layout="nhwc")
    B, nb = 8, 24

    def run(lanes):
        desc = (f"videotestsrc num-buffers={B * nb} pattern=snow pool-size=96 "
                "! video/x-raw,format=RGB,width=224,height=224,framerate=0/1 "
                f"! tensor_converter frames-per-tensor={B} device=0 ! queue max-size-buffers=2 "
                f"! tensor_filter name=f framework=pytorch model={model} input=3:224:224:{B} inputtype=uint8 "
                f"accelerator=true:gpu device=0 custom=hipgraph:true,lanes:{lanes} device-stats=true "
                f"! queue max-size-buffers=4 ! tensor_decoder mode=image_labeling option1={labels} "
                "! tensor_sink name=sink")
        p = nns.parse_launch(desc)
        out = []
        p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes().decode()))
        p.run(timeout=180)
        stamps = [e for e in p.get_by_name("f").get_property("device-stamps").split(",") if e]
        p.stop()
        return out, stamps

    one, st1 = run(1)
    three, st3 = run(3)
    # (image_labeling: one buffer of B newline-separated labels per batch)
    assert len(one) == nb and len(st1) == nb and len(st3) == nb
    assert all(len(x.split("\n")) == B for x in one)
    assert three == one


def test_filter_device_stats(nns, workdir, labels):
    """tensor_filter latency / throughput / device-stamps come from HIP events
    on the element's stream (device time), one record per invoke."""
    import os

    from nnstreamer_amd.models.export import export

    model = export("mobilenet_v2_fused_fp32", os.path.join(workdir, "mbv2_f32_stats.pt"), layout="nhwc")
    desc = ("videotestsrc num-buffers=40 pattern=snow ! video/x-raw,format=RGB,width=224,height=224,framerate=0/1 "
            "! tensor_converter frames-per-tensor=4 device=0 "
            f"! tensor_filter name=f framework=pytorch model={model} input=3:224:224:4 inputtype=uint8 "
            "accelerator=true:gpu device=0 latency=1 throughput=1 device-stats=true "
            f"! tensor_decoder mode=image_labeling option1={labels} ! tensor_sink name=sink")
    p = nns.parse_launch(desc)
    p.run(timeout=120)
    f = p.get_by_name("f")
    stamps = [tuple(int(v) for v in e.split(":")) for e in f.get_property("device-stamps").split(",") if e]
    lat = int(f.get_property("latency"))
    thr = int(f.get_property("throughput"))
    p.stop()
    assert len(stamps) == 10
    ends = [s[0] for s in stamps]
    assert all(b >= a for a, b in zip(ends, ends[1:])), ends
    assert all(0 < s[1] < 1e9 for s in stamps), stamps
    assert lat > 0 and thr > 0


def _ref_string_labels(nns, model, labels, B, absorb):
    """bench.py's reference string at batch B: uint8 frames -> tensor_transform
    (normalisation) -> tensor_filter (fused fp32, hipGraph) -> image_labeling.
    Returns (labels per frame, frames, absorbed-by)."""
    desc = (f"videotestsrc num-buffers={B} pattern=snow pool-size={B} "
            "! video/x-raw,format=RGB,width=224,height=224,framerate=0/1 "
            f"! tee name=t t. ! queue ! tensor_converter frames-per-tensor={B} device=0 "
            "! tensor_transform name=norm mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 "
            f"! queue max-size-buffers=2 ! tensor_filter name=f framework=pytorch model={model} "
            f"input=3:224:224:{B} inputtype=float32 absorb-transform={'true' if absorb else 'false'} "
            "accelerator=true:gpu device=0 custom=hipgraph:true ! queue max-size-buffers=4 "
            f"! tensor_decoder mode=image_labeling option1={labels} ! tensor_sink name=sink "
            f"t. ! queue ! tensor_converter frames-per-tensor={B} ! appsink name=raw")
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes().decode()))
    raw = p.get_by_name("raw")
    p.set_state("playing")
    b = raw.pull(timeout=120)
    assert b is not None
    frames = b.memory(0).numpy("uint8").copy()
    p.wait(timeout=300)
    absorbed = p.get_by_name("norm").get_property("absorbed-by")
    p.stop()
    assert len(out) == 1
    return out[0].split("\n"), frames, absorbed


def test_reference_string_absorbed_at_bench_batch(nns, workdir, labels):
    """The reference pipeline string at the benched batch (512): the filter
    absorbs the tensor_transform into the fused stem's input table; labels
    equal the same string with the transform's own kernel (float32 frames into
    the unfused stem path) and torch.argmax of the plain fp32 model."""
    import os

    from nnstreamer_amd.models.export import export
    from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2

    model = export("mobilenet_v2_fused_fp32", os.path.join(workdir, "mbv2_f32_refstr.pt"), layout="nhwc")
    B = 512
    got, frames, absorbed = _ref_string_labels(nns, model, labels, B, True)
    assert absorbed == "f"
    got_k, frames_k, absorbed_k = _ref_string_labels(nns, model, labels, B, False)
    assert absorbed_k == ""
    assert np.array_equal(frames, frames_k)  # snow is seeded: the same 512 frames
    m = mobilenet_v2(seed=0).cuda().eval()
    x = torch.from_numpy(frames).cuda().view(B, 224, 224, 3).float()
    with torch.no_grad():
        ref = m(((x - 127.5) / 127.5).permute(0, 3, 1, 2)).argmax(1).tolist()
    ref = [f"class_{i}" for i in ref]
    same = sum(a == b for a, b in zip(got, got_k))
    agree = sum(a == b for a, b in zip(got, ref))
    assert same >= B - 2, (same, B)       # two fp32 kernel paths: ties may flip at most a frame or two
    assert agree >= 0.995 * B, (agree, B)


@pytest.mark.parametrize("B", [16, 1])
def test_decoder_argmax_absorbed_in_graph(nns, workdir, labels, B):
    """tensor_filter (fused fp32, hipGraph) ! queue ! tensor_decoder
    mode=image_labeling: the filter captures the decoder's argmax in its graph
    (int32 indices leave the model, runtime/fusion.h ArgmaxConsumer); labels
    equal the pipeline where the decoder runs its own argmax kernel."""
    import os

    from nnstreamer_amd.models.export import export

    model = export("mobilenet_v2_fused_fp32", os.path.join(workdir, "mbv2_f32_argmax.pt"), layout="nhwc")

    def run(absorb):
        desc = (f"videotestsrc num-buffers={B * 3} pattern=snow pool-size=48 "
                "! video/x-raw,format=RGB,width=224,height=224,framerate=0/1 "
                f"! tensor_converter frames-per-tensor={B} device=0 "
                f"! tensor_filter name=f framework=pytorch model={model} input=3:224:224:{B} inputtype=uint8 "
                f"accelerator=true:gpu device=0 custom=hipgraph:true absorb-decoder={'true' if absorb else 'false'} "
                f"! queue max-size-buffers=4 ! tensor_decoder name=dec mode=image_labeling option1={labels} "
                "! tensor_sink name=sink")
        p = nns.parse_launch(desc)
        out = []
        p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes().decode()))
        p.run(timeout=120)
        info = (p.get_by_name("f").get_property("absorbed-decoder"), p.get_by_name("dec").get_property("argmax-by"))
        p.stop()
        return out, info

    a, info = run(True)
    assert info == ("dec", "f")
    b, info_b = run(False)
    assert info_b == ("", "")
    assert len(a) == 3 and a == b
