"""PoseNet (MobileNetV1 backbone, output stride 32, 257x257), random init.

Outputs match the reference's pose_estimation decoder in ``heatmap-offset``
mode (tensordec-pose.c:40-60, 760-800): heatmaps ``17:9:9:B`` and offsets
``34:9:9:B`` -- NHWC ``[B, 9, 9, 17]`` and ``[B, 9, 9, 34]`` float32.
``write_pose_labels`` writes the 17-keypoint connection file (option3).

* ``PoseNetMobileNetV1`` -- plain fp32 oracle.
* ``FusedPoseNet``       -- BN-folded NHWC bf16 on the CDNA4 kernels (the
  whole backbone is depthwise-separable: DW + MFMA PW pairs).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn

from .fused import DW, PW, _fold, input_lut, stem
from .mobilenet_v2 import ConvBNReLU

# (out channels, stride) of the 13 depthwise-separable blocks of MobileNetV1
V1_BLOCKS = [(64, 1), (128, 2), (128, 1), (256, 2), (256, 1), (512, 2), (512, 1), (512, 1), (512, 1), (512, 1),
             (512, 1), (1024, 2), (1024, 1)]
KEYPOINTS = ["nose", "leftEye", "rightEye", "leftEar", "rightEar", "leftShoulder", "rightShoulder", "leftElbow",
             "rightElbow", "leftWrist", "rightWrist", "leftHip", "rightHip", "leftKnee", "rightKnee", "leftAnkle",
             "rightAnkle"]
CONNECTIONS = [[1, 2, 3, 4], [0, 2, 3], [0, 1, 4], [0, 1], [0, 2], [6, 7, 11], [5, 8, 12], [5, 9], [6, 10], [7],
               [8], [5, 12, 13], [6, 11, 14], [11, 15], [12, 16], [13], [14]]


class PoseNetMobileNetV1(nn.Module):
    def __init__(self, keypoints: int = 17):
        super().__init__()
        layers = [ConvBNReLU(3, 32, stride=2)]
        cin = 32
        for cout, s in V1_BLOCKS:
            layers.append(ConvBNReLU(cin, cin, k=3, stride=s, groups=cin))
            layers.append(ConvBNReLU(cin, cout, k=1))
            cin = cout
        self.backbone = nn.Sequential(*layers)
        self.heatmap = nn.Conv2d(1024, keypoints, 1)
        self.offsets = nn.Conv2d(1024, 2 * keypoints, 1)

    def reset_parameters(self, seed: int = 0):
        g = torch.Generator().manual_seed(seed)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                fan_out = m.out_channels * m.kernel_size[0] * m.kernel_size[1] // m.groups
                with torch.no_grad():
                    m.weight.copy_(torch.randn(m.weight.shape, generator=g) * (2.0 / fan_out) ** 0.5)
                    if m.bias is not None:
                        m.bias.zero_()
            elif isinstance(m, nn.BatchNorm2d):
                with torch.no_grad():
                    m.weight.copy_(1.0 + 0.1 * torch.randn(m.weight.shape, generator=g))
                    m.bias.copy_(0.1 * torch.randn(m.bias.shape, generator=g))
                    m.running_mean.copy_(0.1 * torch.randn(m.running_mean.shape, generator=g))
                    m.running_var.copy_(1.0 + 0.1 * torch.rand(m.running_var.shape, generator=g))
        with torch.no_grad():
            self.heatmap.weight.mul_(0.1)
            self.offsets.weight.mul_(0.1)

    def forward(self, x):
        h = self.backbone(x.permute(0, 3, 1, 2))
        return self.heatmap(h).permute(0, 2, 3, 1), self.offsets(h).permute(0, 2, 3, 1)


def posenet(seed: int = 0) -> PoseNetMobileNetV1:
    m = PoseNetMobileNetV1()
    m.reset_parameters(seed)
    return m.eval()


def _padded_pw(conv: nn.Conv2d, precision: str = "bf16") -> PW:
    w = conv.weight.detach().float()
    b = conv.bias.detach().float()
    n = w.shape[0]
    n8 = (n + 7) // 8 * 8
    wp = torch.zeros(n8, w.shape[1], 1, 1)
    wp[:n] = w
    bp = torch.zeros(n8)
    bp[:n] = b
    return PW(wp, bp, act=0, out_f32=True, precision=precision)


class FusedPoseNet(nn.Module):
    """Input [B,257,257,3] f32 NHWC.  Outputs heatmaps [B,9,9,17], offsets [B,9,9,34] (f32)."""

    def __init__(self):
        super().__init__()

    @classmethod
    def from_reference(cls, m: PoseNetMobileNetV1, precision: str = "bf16") -> "FusedPoseNet":
        self = cls()
        m = m.eval()
        self.f32 = precision == "fp32"
        stem: ConvBNReLU = m.backbone[0]
        w, b = _fold(stem[0], stem[1])
        self.register_buffer("stem_w", w.permute(2, 3, 1, 0).contiguous())
        self.register_buffer("stem_b", b.contiguous())
        self.register_buffer("in_lut", input_lut(-127.5, 127.5))  # uint8 input table (absorbable transform)
        dws, pws = [], []
        layers = list(m.backbone)[1:]
        for i in range(0, len(layers), 2):
            d: ConvBNReLU = layers[i]
            p: ConvBNReLU = layers[i + 1]
            dws.append(DW(*_fold(d[0], d[1]), stride=int(d[0].stride[0]), precision=precision))
            pws.append(PW(*_fold(p[0], p[1]), act=1, precision=precision))
        self.dws = nn.ModuleList(dws)
        self.pws = nn.ModuleList(pws)
        self.heat = _padded_pw(m.heatmap, precision)
        self.offs = _padded_pw(m.offsets, precision)
        self.k = int(m.heatmap.out_channels)
        return self

    def forward(self, x: torch.Tensor):
        h = stem(x, self.stem_w, self.stem_b, self.in_lut, self.f32)
        for d, p in zip(self.dws, self.pws):
            h = p(d(h))
        if self.f32 and h.is_cuda:
            # both 1x1 heads in one grouped GEMM launch, exact columns (no slice copies)
            o = torch.ops.nnsx.pw_conv_group([h, h], [self.heat.wt, self.offs.wt], [self.heat.bias, self.offs.bias],
                                             [self.k, 2 * self.k], [0, 0])
            return o[0], o[1]
        hm = self.heat(h)[..., : self.k].contiguous()
        of = self.offs(h)[..., : 2 * self.k].contiguous()
        return hm, of


def fused_posenet(seed: int = 0, precision: str = "bf16") -> FusedPoseNet:
    return FusedPoseNet.from_reference(posenet(seed), precision).eval()


def write_pose_labels(path: str) -> str:
    with open(path, "w") as f:
        for name, conn in zip(KEYPOINTS, CONNECTIONS):
            f.write(" ".join([name] + [str(c) for c in conn]) + "\n")
    return path
