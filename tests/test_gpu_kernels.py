"""Numerics of the hand-written CDNA4 kernels against plain PyTorch fp32/fp64
references (run on the MI355X box)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

TYPES = {  # nnsx DType ordinal -> torch dtype
    0: torch.int32, 2: torch.int16, 4: torch.int8, 5: torch.uint8,
    6: torch.float64, 7: torch.float32, 8: torch.int64, 10: torch.float16, 12: torch.bfloat16,
}


def _stream():
    return torch.cuda.current_stream().cuda_stream


@pytest.mark.parametrize("n", [1, 7, 8, 1000, 150528, 3 * 224 * 224 * 4 + 5])
def test_arith_u8_to_f32_normalize(nns, n):
    x = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda")
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    ops = [(0, -127.5, -127, 0.0, -1), (2, 127.5, 127, 0.0, -1)]
    nns.kernels.arith(x.data_ptr(), 5, out.data_ptr(), 7, n, ops, 1, 0, _stream())
    ref = (x.float() + (-127.5)) / 127.5
    torch.testing.assert_close(out, ref, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("in_t,out_t", [(5, 7), (7, 5), (7, 12), (12, 7), (0, 7), (7, 10), (4, 0), (6, 7)])
def test_typecast_pairs(nns, in_t, out_t):
    n = 4099
    src = (torch.randn(n, dtype=torch.float64, device="cuda") * 50)
    if not TYPES[in_t].is_floating_point:
        info = torch.iinfo(TYPES[in_t])
        src = src.clamp(info.min, info.max)
    x = src.to(TYPES[in_t])
    out = torch.empty(n, dtype=TYPES[out_t], device="cuda")
    nns.kernels.arith(x.data_ptr(), in_t, out.data_ptr(), out_t, n, [], 1, 0, _stream())
    if TYPES[out_t].is_floating_point:
        ref = x.to(torch.float64).to(TYPES[out_t])
        torch.testing.assert_close(out, ref)
    else:
        # C conversion semantics: truncate toward zero, out-of-range wraps modulo 2^bits
        bits = torch.iinfo(TYPES[out_t]).bits
        ref = x.to(torch.float64).trunc().to(torch.int64) % (1 << bits)
        torch.testing.assert_close(out.to(torch.int64) % (1 << bits), ref)


def test_arith_int_wraps_like_c(nns):
    x = torch.tensor([100, 120, -128, 5], dtype=torch.int8, device="cuda")
    out = torch.empty_like(x)
    nns.kernels.arith(x.data_ptr(), 4, out.data_ptr(), 4, 4, [(0, 100.0, 100, 0.0, -1)], 1, 0, _stream())
    ref = ((x.to(torch.int64) + 100 + 128) % 256 - 128).to(torch.int8)
    assert torch.equal(out, ref)


def test_arith_per_channel(nns):
    # 3:4:2:1 tensor, per-channel add on channel 1 only (dim 0 is the channel)
    x = torch.arange(24, dtype=torch.float32, device="cuda")
    out = torch.empty_like(x)
    nns.kernels.arith(x.data_ptr(), 7, out.data_ptr(), 7, 24, [(0, 10.0, 10, 0.0, 1)], 1, 3, _stream())
    ref = x.clone().view(-1, 3)
    ref[:, 1] += 10
    torch.testing.assert_close(out, ref.view(-1))


def test_clamp(nns):
    x = torch.randn(5000, device="cuda") * 10
    out = torch.empty_like(x)
    nns.kernels.arith(x.data_ptr(), 7, out.data_ptr(), 7, 5000, [(3, -1.5, 0, 2.5, -1)], 1, 0, _stream())
    torch.testing.assert_close(out, x.clamp(-1.5, 2.5))


@pytest.mark.parametrize("dims,perm", [
    ([3, 224, 224, 1], [1, 2, 0, 3]),
    ([3, 224, 224, 4], [1, 2, 0, 3]),
    ([64, 32, 5, 2], [2, 0, 1, 3]),
    ([5, 7, 11, 3], [0, 2, 1, 3]),
    ([40, 48, 2, 1], [1, 0, 2, 3]),
])
def test_permute(nns, dims, perm):
    n = int(np.prod(dims))
    x = torch.randn(n, device="cuda")
    out = torch.empty_like(x)
    nns.kernels.permute(x.data_ptr(), out.data_ptr(), 4, dims, perm, _stream())
    # reference in torch (reverse the innermost-first dims to get row-major shape)
    t = x.view(dims[::-1])
    # out.dim[k] = in.dim[perm[k]] ; torch axis of nnsx axis a is (rank-1-a)
    r = len(dims)
    order = [r - 1 - perm[k] for k in reversed(range(r))]
    ref = t.permute(order).contiguous().view(-1)
    torch.testing.assert_close(out, ref)


@pytest.mark.parametrize("es,dims,perm", [
    (4, [3, 5, 7, 11, 13], [3, 1, 4, 0, 2]),
    (1, [4, 6, 1, 9, 2], [2, 4, 0, 3, 1]),
    (2, [33, 2, 65, 3], [2, 3, 0, 1]),
    (8, [7, 40, 3, 2, 5, 3], [5, 4, 1, 0, 3, 2]),
    (4, [16, 9, 8, 5], [0, 2, 1, 3]),        # innermost kept: row copies
    (1, [3, 64, 64, 2, 2], [2, 1, 0, 4, 3]),
    (4, [2, 3, 4, 5, 6, 7, 2, 1], [7, 6, 5, 4, 3, 2, 1, 0]),
])
def test_permute_general(nns, es, dims, perm):
    """every permutation class: the tiled (axis 0 <-> output-innermost axis
    through LDS, batch axes decomposed per workgroup) and row-copy kernels"""
    dt = {1: torch.uint8, 2: torch.int16, 4: torch.float32, 8: torch.float64}[es]
    n = int(np.prod(dims))
    x = (torch.rand(n, device="cuda") * 100).to(dt)
    out = torch.zeros_like(x)
    nns.kernels.permute(x.data_ptr(), out.data_ptr(), es, dims, perm, _stream())
    r = len(dims)
    order = [r - 1 - perm[k] for k in reversed(range(r))]
    ref = x.view(dims[::-1]).permute(order).contiguous().view(-1)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("t", [7, 5, 12])
def test_argmax_rows_first_max_wins(nns, t):
    rows, n = 33, 1001
    x = (torch.randn(rows, n, device="cuda") * 5).to(TYPES[t])
    if not x.is_floating_point():
        x = x.clamp(max=200)
    x[3, 10] = x[3].max() + 1
    x[3, 20] = x[3, 10]
    out = torch.empty(rows, dtype=torch.int32, device="cuda")
    nns.kernels.argmax_rows(x.data_ptr(), t, n, rows, out.data_ptr(), _stream())
    ref = torch.tensor([int(np.argmax(r)) for r in x.float().cpu().numpy()], dtype=torch.int32)
    assert torch.equal(out.cpu(), ref)
    assert int(out[3]) == 10


@pytest.mark.parametrize("per_ch", [False, True])
@pytest.mark.parametrize("mode", [0, 1])
def test_stand(nns, per_ch, mode):
    C, n = 3, 3 * 50 * 40
    x = torch.rand(n, device="cuda") * 255
    out = torch.empty_like(x)
    ws = torch.empty(nns.kernels.stand_workspace_bytes(C), dtype=torch.uint8, device="cuda")
    nns.kernels.stand(x.data_ptr(), 7, out.data_ptr(), 7, n, C, mode, per_ch, ws.data_ptr(), _stream())
    xd = x.double()
    if per_ch:
        v = xd.view(-1, C)
        mean = v.mean(0)
        std = v.std(0, unbiased=False)
        ref = ((v - mean) / std).abs() if mode == 0 else (v - mean)
        ref = ref.view(-1)
    else:
        mean, std = xd.mean(), xd.std(unbiased=False)
        ref = ((xd - mean) / std).abs() if mode == 0 else xd - mean
    torch.testing.assert_close(out.double(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("C", [1, 3, 7, 300])
def test_stand_deterministic_large(nns, C):
    """The device stand reduction is a fixed-order two-level sum (no atomics):
    bitwise-identical outputs run to run, at sizes where the reduction spans
    every level-1 block (and C > 256, the channel-loop path)."""
    n = C * 200_003
    x = (torch.rand(n, device="cuda") * 255).contiguous()
    ws = torch.empty(nns.kernels.stand_workspace_bytes(C), dtype=torch.uint8, device="cuda")
    outs = []
    for _ in range(3):
        out = torch.empty_like(x)
        nns.kernels.stand(x.data_ptr(), 7, out.data_ptr(), 7, n, C, 0, True, ws.data_ptr(), _stream())
        torch.cuda.synchronize()
        outs.append(out)
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
    v = x.double().view(-1, C)
    ref = ((v - v.mean(0)) / v.std(0, unbiased=False)).abs().view(-1)
    torch.testing.assert_close(outs[0].double(), ref, rtol=1e-5, atol=1e-4)
