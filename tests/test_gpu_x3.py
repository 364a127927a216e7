"""Split-bf16 ("x3") fp32 products (csrc/kernels/mbv2_f32.hip, split_x3 /
mfma_x3): every operand split exactly into three bf16 parts, six cross
products on v_mfma_f32_16x16x32_bf16, 32-k partials added in fp32.

The method counts as fp32 only if its error against an fp64 oracle is no
worse than the native fp32 MFMA kernel's on the same operands -- max and mean
relative error, shape by shape (the reference computes in float32:
tensor_filter_pytorch.cc:517-536).  Each test runs both methods
(torch.ops.nnsx.set_f32_math) on the same data and compares their errors."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def method():
    prev = torch.ops.nnsx.f32_math()
    yield lambda m: torch.ops.nnsx.set_f32_math(m)
    torch.ops.nnsx.set_f32_math(prev)


def _errs(y, ref):
    """(max, mean) of |y - ref| / scale, scale = max(1, max |ref|)"""
    d = (y.double().cpu() - ref).abs()
    scale = max(1.0, ref.abs().max().item())
    return d.max().item() / scale, d.mean().item() / scale


def _both(method, fn, ref, differ=False):
    """errors of the native and the x3 method on the same call; differ: the x3
    path must really run (its result is not the native one bit for bit)"""
    method("fp32")
    y_nat = fn()
    e_nat = _errs(y_nat, ref)
    method("x3")
    y = fn()
    e_x3 = _errs(y, ref)
    if differ:
        assert not torch.equal(y, y_nat), "x3 method did not run (same bits as native)"
    return e_nat, e_x3, y


def _x3_expected(method, stride, H, cin, hid, cout, B):
    method("x3")
    return torch.ops.nnsx.ir_method_f32(stride, H, H, cin, hid, cout, B, 1) == "x3"


GEMM_SHAPES = [(1000, 16, 96), (777, 24, 144), (4096, 144, 24), (6272, 320, 1280), (128, 1280, 1000),
               (130, 960, 160), (6272, 160, 960), (6272, 960, 320), (25088, 320, 1280), (4225, 64, 128),
               (1089, 512, 1024)]


@pytest.mark.parametrize("M,K,N", GEMM_SHAPES)
@pytest.mark.parametrize("act,use_res,dist", [(1, False, "relu6"), (0, True, "relu6"), (0, False, "normal")])
def test_x3_gemm_no_worse_than_native(nns, method, M, K, N, act, use_res, dist):
    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device="cuda")
    if dist == "relu6":  # MobileNet activations: ReLU6 outputs, many zeros, some clamped
        x = (x * 2).clamp(0, 6)
    npad, kpad = (N + 15) // 16 * 16, (K + 7) // 8 * 8
    wt = torch.zeros(npad, kpad, device="cuda")
    wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
    bias = torch.randn(npad, device="cuda") * 0.1
    res = torch.randn(M, N, device="cuda") if use_res else None
    ref = x.double().cpu() @ wt[:N, :K].double().cpu().t() + bias[:N].double().cpu()
    if use_res:
        ref = ref + res.double().cpu()
    if act == 1:
        ref = ref.clamp(0, 6)
    (nat_max, nat_mean), (x3_max, x3_mean), y = _both(
        method, lambda: torch.ops.nnsx.pw_conv(x, wt, bias, res, N, act, True), ref, differ=True)
    assert x3_max <= nat_max and x3_mean <= nat_mean, (nat_max, x3_max, nat_mean, x3_mean)
    # and deterministic (fixed k order; split-K slabs added in order)
    assert torch.equal(y, torch.ops.nnsx.pw_conv(x, wt, bias, res, N, act, True))


def test_x3_gemm_identity_asymmetric(nns, method):
    """A = I with an asymmetric B: a transposed fragment or a k permutation
    that differs between the operands shows as wrong elements, exactly"""
    method("x3")
    M, K, N = 192, 64, 64
    x = torch.arange(M * K, device="cuda", dtype=torch.float32).view(M, K).remainder(13) - 6
    x = x + torch.arange(K, device="cuda", dtype=torch.float32) * 2 ** -12  # mid / lo parts non-zero
    wt = torch.eye(64, device="cuda")
    y = torch.ops.nnsx.pw_conv(x, wt, torch.zeros(64, device="cuda"), None, N, 0, True)
    torch.testing.assert_close(y, x, rtol=0, atol=0)


def test_x3_split_is_exact_for_fp32_operands(nns, method):
    """x = hi + mid + lo exactly for fp32 inputs across the exponent range the
    engine sees: a one-hot weight row reproduces each input bit for bit"""
    method("x3")
    torch.manual_seed(0)
    M, K, N = 256, 32, 32
    mag = torch.pow(2.0, torch.randint(-30, 30, (M, K), device="cuda").float())
    x = torch.randn(M, K, device="cuda") * mag
    wt = torch.eye(32, device="cuda")
    y = torch.ops.nnsx.pw_conv(x, wt, torch.zeros(32, device="cuda"), None, N, 0, True)
    torch.testing.assert_close(y, x, rtol=0, atol=0)


@pytest.fixture
def x3_cache():
    prev = torch.ops.nnsx.x3_weight_cache(True)
    yield lambda on: torch.ops.nnsx.x3_weight_cache(on)
    torch.ops.nnsx.x3_weight_cache(prev)


@pytest.mark.parametrize("tile", [0, 64064, 128064, 64128, 128128, 128192])
@pytest.mark.parametrize("M,K,N", [(6272, 960, 320), (4225, 64, 128), (1000, 24, 144), (130, 1280, 1000)])
def test_x3_presplit_weights_match_per_tile_split(nns, method, x3_cache, tile, M, K, N):
    """The pre-split weight path (weights split once, staged as bf16 parts) and
    the per-tile split give the same bits: same RNE parts, same products"""
    method("x3")
    torch.manual_seed(M + K + N + tile)
    x = (torch.randn(M, K, device="cuda") * 2).clamp(0, 6)
    npad, kpad = (N + 15) // 16 * 16, (K + 7) // 8 * 8
    wt = torch.zeros(npad, kpad, device="cuda")
    wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
    bias = torch.randn(npad, device="cuda") * 0.1
    x3_cache(False)
    y0 = torch.ops.nnsx.pw_conv_f32_tile(x, wt, bias, None, N, 1, tile)
    x3_cache(True)
    y1 = torch.ops.nnsx.pw_conv_f32_tile(x, wt, bias, None, N, 1, tile)
    y2 = torch.ops.nnsx.pw_conv_f32_tile(x, wt, bias, None, N, 1, tile)  # (cache hit)
    assert torch.equal(y0, y1) and torch.equal(y1, y2)


def test_x3_presplit_weights_follow_in_place_updates(nns, method, x3_cache):
    """An in-place change of the weights is split again (version check), and a
    new weight tensor is never served another's parts"""
    method("x3")
    torch.manual_seed(5)
    x = torch.randn(2048, 96, device="cuda")
    wt = torch.randn(160, 96, device="cuda") / 10
    bias = torch.zeros(160, device="cuda")
    y1 = torch.ops.nnsx.pw_conv(x, wt, bias, None, 160, 0, True)
    wt.mul_(2)
    y2 = torch.ops.nnsx.pw_conv(x, wt, bias, None, 160, 0, True)
    torch.testing.assert_close(y2, 2 * y1, rtol=1e-6, atol=1e-6)
    wt2 = torch.randn(160, 96, device="cuda") / 10
    ref = (x.double() @ wt2.double().t()).float()
    torch.testing.assert_close(torch.ops.nnsx.pw_conv(x, wt2, bias, None, 160, 0, True), ref, rtol=1e-5, atol=1e-5)


def test_x3_presplit_weights_grouped_and_pooled(nns, method, x3_cache):
    """pw_conv_group (PoseNet heads), pw_conv_pool (head + pool), pw_conv_into
    and pw_conv_rowbias: the same bits with and without the pre-split weights"""
    method("x3")
    torch.manual_seed(9)
    xs = [torch.randn(4, 17, 17, 64, device="cuda").clamp(0, 6), torch.randn(4, 9, 9, 128, device="cuda").clamp(0, 6)]
    wts = [torch.randn(48, 64, device="cuda") / 8, torch.randn(32, 128, device="cuda") / 11]
    bs = [torch.randn(48, device="cuda"), torch.randn(32, device="cuda")]
    xp = torch.randn(64, 7, 7, 320, device="cuda").clamp(0, 6)
    wp = torch.randn(1280, 320, device="cuda") / 18
    bp = torch.randn(1280, device="cuda")
    rb = torch.randn(4, 256, device="cuda")
    wr = torch.randn(256, 64, device="cuda") / 8

    def run():
        out = torch.zeros(4, 17 * 17 * 2 + 5, 24, device="cuda")
        torch.ops.nnsx.pw_conv_into(xs[0], wts[0], bs[0], out, 5, 48, 0)
        return (torch.ops.nnsx.pw_conv_group(xs, wts, bs, [48, 32], [0, 1])
                + [torch.ops.nnsx.pw_conv_pool(xp, wp, bp, 1280, 1), out,
                   torch.ops.nnsx.pw_conv_rowbias(xs[0], wr, rb, 256, 1)])
    x3_cache(False)
    a = run()
    x3_cache(True)
    b = run()
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("B,H", [(9, 7), (64, 7), (171, 7)])
def test_x3_head_pool_no_worse_than_native(nns, method, B, H):
    torch.manual_seed(B * 7 + H)
    K, N = 320, 1280
    x = (torch.randn(B, H, H, K, device="cuda") * 2).clamp(0, 6)
    wt = torch.randn(N, K, device="cuda") / K ** 0.5
    bias = torch.randn(N, device="cuda") * 0.1
    ref = (x.double().cpu() @ wt.double().cpu().t() + bias.double().cpu()).clamp(0, 6).mean((1, 2))
    (nat_max, nat_mean), (x3_max, x3_mean), _ = _both(
        method, lambda: torch.ops.nnsx.pw_conv_pool(x, wt, bias, N, 1), ref)
    # (the pooled mean's own fp32 sums, shared by both methods, set the max error)
    assert x3_mean <= nat_mean and x3_max <= 1.1 * nat_max, (nat_max, x3_max, nat_mean, x3_mean)


def _ir_weights(cin, hid, cout, seed):
    from nnstreamer_amd.models.fused import x3_split

    torch.manual_seed(seed)
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
    we3 = x3_split(we[:, :cin].cpu(), hid, (cin + 31) // 32 * 32).cuda()
    wp3 = x3_split(wp[:cout].cpu(), (cout + 31) // 32 * 32, hid).cuda()
    return we, be, wd, bd, wp, bp, we3, wp3


from test_gpu_mbv2_f32 import IR_F32_SHAPES, _ir_ref64  # noqa: E402


@pytest.mark.parametrize("H,cin,hid,cout,stride,has_expand", [s for s in IR_F32_SHAPES if s[5]])
@pytest.mark.parametrize("B", [3, 1])
def test_x3_ir_block_no_worse_than_native(nns, method, H, cin, hid, cout, stride, has_expand, B):
    """every fused inverted-residual shape of the fp32 suite: the x3 kernel
    (irw_x3) against the native one on the same data, both vs fp64"""
    we, be, wd, bd, wp, bp, we3, wp3 = _ir_weights(cin, hid, cout, H * 7 + cin + hid)
    x = torch.randn(B, H, H, cin, device="cuda")
    residual = stride == 1 and cin == cout
    ref = _ir_ref64(x, we, be, wd, bd, wp, bp, stride, cout, True, residual)

    def run():
        return torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, residual, 1, None, we3, wp3)

    (nat_max, nat_mean), (x3_max, x3_mean), y = _both(
        method, run, ref, differ=_x3_expected(method, stride, H, cin, hid, cout, B))
    # the project sums 16-channel partials: max errors sit at the fp32 rounding
    # of the output; allow 10 % on the max, none on the mean
    assert x3_mean <= nat_mean and x3_max <= 1.1 * nat_max, (nat_max, x3_max, nat_mean, x3_mean)
    assert x3_max < 5e-5
    assert torch.equal(y, run())


@pytest.mark.parametrize("H,cin,hid,cout,stride", [(7, 160, 960, 160, 1), (14, 96, 576, 160, 2),
                                                    (14, 64, 384, 64, 1), (28, 32, 192, 64, 2)])
@pytest.mark.parametrize("B", [1, 8, 128])
def test_x3_ir_block_hidden_parts(nns, method, H, cin, hid, cout, stride, B):
    """small batches split the hidden channels over workgroups (slabs, in-launch
    combine with the ticket buffer, or the reduce launch): bitwise repeatable,
    no worse than native"""
    we, be, wd, bd, wp, bp, we3, wp3 = _ir_weights(cin, hid, cout, cin + hid + B)
    x = torch.randn(B, H, H, cin, device="cuda")
    res = stride == 1 and cin == cout
    tickets = torch.zeros(768, dtype=torch.int32, device="cuda")
    ref = _ir_ref64(x, we, be, wd, bd, wp, bp, stride, cout, True, res)

    def run():
        return torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res, 1, tickets, we3, wp3)

    (nat_max, nat_mean), (x3_max, x3_mean), y = _both(
        method, run, ref, differ=_x3_expected(method, stride, H, cin, hid, cout, B))
    assert x3_mean <= nat_mean and x3_max <= 1.1 * nat_max, (nat_max, x3_max, nat_mean, x3_mean)
    for _ in range(2):
        assert torch.equal(y, run())


@pytest.mark.parametrize("B", [128, 3, 1])
def test_x3_ir_expand_dw(nns, method, B):
    """the expand + depthwise kernel (7x7 160 -> 960: the x3 twin is the default)"""
    import torch.nn.functional as F

    cin, hid, H = 160, 960, 7
    we, be, wd, bd, _, _, we3, _ = _ir_weights(cin, hid, 16, B)
    x = torch.randn(B, H, H, cin, device="cuda")
    h = (x.double().cpu() @ we.double().cpu().t() + be.double().cpu()).clamp(0, 6)
    ref = F.conv2d(h.permute(0, 3, 1, 2), wd.double().cpu().view(3, 3, hid).permute(2, 0, 1).unsqueeze(1),
                   bd.double().cpu(), padding=1, groups=hid).clamp(0, 6).permute(0, 2, 3, 1)
    (nat_max, nat_mean), (x3_max, x3_mean), _ = _both(
        method, lambda: torch.ops.nnsx.ir_expand_dw(x, we, be, wd, bd, 1, 1, we3), ref)
    assert x3_mean <= nat_mean and x3_max <= 1.1 * nat_max, (nat_max, x3_max, nat_mean, x3_mean)
