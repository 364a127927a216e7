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


def test_posenet_fp32_fused_matches_torch_fp32():
    m = posenet.posenet(seed=3).cuda().eval()
    f = torch.jit.script(posenet.FusedPoseNet.from_reference(posenet.posenet(seed=3), "fp32").cuda().eval())
    x = _u8(4, 257, 2)
    with torch.no_grad():
        fh, fo = f(x)
        h, o = m((x.float() - 127.5) / 127.5)
    assert _rel(fh, h) < 1e-3 and _rel(fo, o) < 1e-3, (_rel(fh, h), _rel(fo, o))
