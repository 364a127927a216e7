"""MobileNetV2 (Sandler et al. 2018), hand-written (torchvision is absent).

Two forms are provided:

* ``MobileNetV2`` -- the plain training-style definition (Conv + BatchNorm +
  ReLU6), random-init.  It is the fp32 numerics oracle for the fused engine.
* ``FusedMobileNetV2`` (see ``fused.py``) -- the inference form the framework
  actually runs on MI355X: BN folded into the conv weights, NHWC bf16
  activations, every conv lowered onto the hand-written CDNA4 kernels in
  ``csrc/kernels/mbv2_*.hip``.

The reference runs MobileNet through ``tensor_filter framework=pytorch``
(``ext/nnstreamer/tensor_filter/tensor_filter_pytorch.cc:197-237``) with the
model loaded from a TorchScript file; ``export_torchscript`` produces such a
file from random-init weights so the same pipeline strings work here.
"""
from __future__ import annotations

import torch
import torch.nn as nn

# (expansion t, output channels c, repeats n, first stride s) -- the paper's Table 2.
INVERTED_RESIDUAL_SETTING = [
    (1, 16, 1, 1),
    (6, 24, 2, 2),
    (6, 32, 3, 2),
    (6, 64, 4, 2),
    (6, 96, 3, 1),
    (6, 160, 3, 2),
    (6, 320, 1, 1),
]


def _make_divisible(v: float, divisor: int = 8) -> int:
    new_v = max(divisor, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class ConvBNReLU(nn.Sequential):
    def __init__(self, cin: int, cout: int, k: int = 3, stride: int = 1, groups: int = 1, act: bool = True):
        layers = [
            nn.Conv2d(cin, cout, k, stride, (k - 1) // 2, groups=groups, bias=False),
            nn.BatchNorm2d(cout),
        ]
        if act:
            layers.append(nn.ReLU6(inplace=True))
        super().__init__(*layers)


class InvertedResidual(nn.Module):
    def __init__(self, cin: int, cout: int, stride: int, expand: int):
        super().__init__()
        hidden = int(round(cin * expand))
        self.use_res = stride == 1 and cin == cout
        self.stride = stride
        self.expand = expand
        layers = []
        if expand != 1:
            layers.append(ConvBNReLU(cin, hidden, k=1))
        layers.append(ConvBNReLU(hidden, hidden, k=3, stride=stride, groups=hidden))
        layers.append(ConvBNReLU(hidden, cout, k=1, act=False))
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        if self.use_res:
            return x + self.conv(x)
        return self.conv(x)


class MobileNetV2(nn.Module):
    """Input NCHW float, 224x224.  Output logits [N, num_classes]."""

    def __init__(self, num_classes: int = 1000, width_mult: float = 1.0):
        super().__init__()
        cin = _make_divisible(32 * width_mult)
        self.last_channel = _make_divisible(1280 * max(1.0, width_mult))
        features = [ConvBNReLU(3, cin, stride=2)]
        for t, c, n, s in INVERTED_RESIDUAL_SETTING:
            cout = _make_divisible(c * width_mult)
            for i in range(n):
                features.append(InvertedResidual(cin, cout, s if i == 0 else 1, t))
                cin = cout
        features.append(ConvBNReLU(cin, self.last_channel, k=1))
        self.features = nn.Sequential(*features)
        self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(self.last_channel, num_classes))
        self.reset_parameters()

    def reset_parameters(self, seed: int | None = None):
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan_out = m.out_channels * m.kernel_size[0] * m.kernel_size[1] // m.groups
                with torch.no_grad():
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / fan_out) ** 0.5)
            elif isinstance(m, nn.BatchNorm2d):
                with torch.no_grad():
                    # non-trivial running stats so BN folding is actually exercised
                    m.weight.copy_(1.0 + 0.1 * torch.randn(m.weight.shape, generator=g))
                    m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=g))
                    m.running_mean.copy_(0.1 * torch.randn(m.running_mean.shape, generator=g))
                    m.running_var.copy_(1.0 + 0.1 * torch.rand(m.running_var.shape, generator=g))
            elif isinstance(m, nn.Linear):
                with torch.no_grad():
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * 0.01)
                    m.bias.zero_()

    def forward(self, x):
        x = self.features(x)
        x = x.mean((2, 3))
        return self.classifier(x)


def mobilenet_v2(num_classes: int = 1000, seed: int = 0) -> MobileNetV2:
    m = MobileNetV2(num_classes)
    m.reset_parameters(seed)
    return m.eval()
