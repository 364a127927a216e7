"""Load-time lowering of plain TorchScript models onto the nnsx kernels
(csrc/filter/torch_lower.cc) -- what tensor_filter framework=pytorch does to a
user's model on a GPU.  On CPU the lowered graph runs the same torch.ops.nnsx
ops' CPU implementations, so the pass itself (pattern matching, layouts,
weight re-layout, residuals, fallbacks) is checked here against the original
TorchScript model.  Reference: the filter runs whatever torch::jit::load
returns (tensor_filter_pytorch.cc:205-230, invoke :517-557)."""
import os

import pytest
import torch
import torch.nn as nn


def _lower(nns, tmp_path, model, name):
    src = os.path.join(tmp_path, f"{name}.pt")
    dst = os.path.join(tmp_path, f"{name}_low.pt")
    torch.jit.script(model.eval()).save(src)
    rep = nns._C.lower_torchscript(src, dst, -1)
    return rep, torch.jit.load(src).eval(), torch.jit.load(dst).eval()


def _kinds(m):
    out = {}
    for n in m.graph.nodes():
        out[n.kind()] = out.get(n.kind(), 0) + 1
    return out


@pytest.mark.parametrize("layout", ["nhwc", "nchw"])
def test_plain_mobilenet_v2_lowers_whole(nns, tmp_path, layout):
    from nnstreamer_amd.models.export import build_model

    rep, a, b = _lower(nns, tmp_path, build_model("mobilenet_v2", seed=3, layout=layout), f"mbv2_{layout}")
    assert rep.startswith("52/52 convs + 1 linear"), rep
    assert "16 fused inverted residuals" in rep and "stem + block 1 fused" in rep and "head + pool fused" in rep
    k = _kinds(b)
    assert k.get("nnsx::ir_block_any") == 16 and k.get("nnsx::stem_ir1_any") == 1
    assert k.get("nnsx::pw_conv_pool") == 1 and k.get("nnsx::pw_conv") == 1
    assert not any(s.startswith("aten::conv") for s in k), k
    torch.manual_seed(0)
    x = torch.randn(3, 224, 224, 3) if layout == "nhwc" else torch.randn(3, 3, 224, 224)
    with torch.no_grad():
        ya, yb = a(x), b(x)
    assert ya.shape == yb.shape
    assert (ya - yb).abs().max().item() <= 1e-4 * max(1.0, ya.abs().max().item())
    assert torch.equal(ya.argmax(1), yb.argmax(1))


def test_lowered_uint8_input_through_table(nns, tmp_path):
    """the lowered model gets an in_lut table: uint8 frames through it equal
    the original model on the table's float values (what an absorbed
    tensor_transform feeds)"""
    from nnstreamer_amd.models.export import build_model

    _, a, b = _lower(nns, tmp_path, build_model("mobilenet_v2", seed=4, layout="nhwc"), "mbv2_u8")
    lut = (torch.arange(256, dtype=torch.float32) - 127.5) / 127.5
    b.in_lut.copy_(lut)
    x = torch.randint(0, 256, (2, 224, 224, 3), dtype=torch.uint8)
    with torch.no_grad():
        ya = a(lut[x.long()])
        yb = b(x)
    assert (ya - yb).abs().max().item() <= 1e-4 * max(1.0, ya.abs().max().item())


class _Mixed(nn.Module):
    """layers the engine has (1x1, depthwise, ReLU6, residual, linear) between
    layers it has not (5x5 conv, max pool, GELU, sigmoid)"""

    def __init__(self):
        super().__init__()
        self.c5 = nn.Conv2d(3, 16, 5, padding=2)
        self.pw = nn.Conv2d(16, 32, 1)
        self.dw = nn.Conv2d(32, 32, 3, padding=1, groups=32)
        self.pj = nn.Conv2d(32, 16, 1)
        self.pool = nn.MaxPool2d(2)
        self.head = nn.Conv2d(16, 24, 1)
        self.fc = nn.Linear(24, 12)

    def forward(self, x):
        h = torch.nn.functional.gelu(self.c5(x))
        y = self.pj(torch.clamp(self.dw(torch.clamp(self.pw(h), 0.0, 6.0)), 0.0, 6.0))
        h = self.pool(h + y)
        h = torch.relu(self.head(h)).mean((2, 3))
        return torch.sigmoid(self.fc(h))


def test_partially_matched_model_runs_unchanged(nns, tmp_path):
    torch.manual_seed(5)
    rep, a, b = _lower(nns, tmp_path, _Mixed(), "mixed")
    assert "1 fused inverted residuals" in rep and "+ 1 linear" in rep, rep
    k = _kinds(b)
    assert k.get("aten::conv2d") == 1 and k.get("aten::max_pool2d") == 1 and k.get("aten::gelu") == 1, k
    x = torch.randn(2, 3, 20, 20)
    with torch.no_grad():
        ya, yb = a(x), b(x)
    assert (ya - yb).abs().max().item() < 1e-5


def test_unmatched_model_left_alone(nns, tmp_path):
    m = nn.Sequential(nn.Conv2d(3, 8, 7, stride=3), nn.Tanh(), nn.Flatten())
    rep, a, b = _lower(nns, tmp_path, m, "unmatched")
    assert rep.startswith("not lowered"), rep
    x = torch.randn(1, 3, 16, 16)
    with torch.no_grad():
        assert torch.equal(a(x), b(x))
