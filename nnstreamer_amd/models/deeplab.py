"""DeepLabV3-MobileNetV2 (output stride 16) for 513x513 segmentation, random init.

Output layout is what the reference's image_segment decoder consumes in
``tflite-deeplab`` mode (tensordec-imagesegment.c:545-560): per-pixel label
scores with labels innermost, ``21:513:513:B`` -- i.e. an NHWC
``[B, 513, 513, 21]`` float32 tensor.

Backbone: MobileNetV2 features 0..17 with the last stride-2 stage turned into
stride 1 + dilation 2 (33x33 at 513 input).  Head: the mobile ASPP variant
(1x1 branch + image-pooling branch, concat, 1x1 projection, 1x1 classifier)
and a bilinear (align_corners) upsample back to the input size.

* ``DeepLabV3MobileNetV2`` -- plain fp32 oracle (NCHW internally).
* ``FusedDeepLabV3``       -- BN-folded NHWC bf16 / fp32 on the CDNA4 kernels
  (dilated depthwise via ``nnsx::dw_conv(..., dilation)``).  fp32 head: the
  image-pooling branch is constant over space, so ``project(cat[a, p])`` is
  one GEMM on ``a`` with a per-image bias ``W_p . p + b`` (``pw_conv_rowbias``,
  no concat); the classifier writes the 21 labels straight into a contiguous
  ``[B, 33, 33, 21]`` map (``pw_conv_into``); the resize is the hand-written
  NHWC bilinear kernel (``nnsx::upsample_bilinear``).
* ``lowres=True`` (model names ``deeplab_fused_lowres*``) -- the model ships the
  33x33 logits and the pipeline's decoder resizes them
  (``tensor_decoder mode=image_segment option1=tflite-deeplab option3=513:513``:
  upsample + argmax + colour map in one pass, kernels/vision.hip), so the
  513x513x21 score map (22 MB per frame) never exists.  Same decoded frames.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .fused import PW, Block, StemBlock1, _fold, input_lut
from .mobilenet_v2 import ConvBNReLU, InvertedResidual, MobileNetV2


class DeepLabV3MobileNetV2(nn.Module):
    def __init__(self, num_classes: int = 21, out_size: int = 513):
        super().__init__()
        feats = list(MobileNetV2().features)[:-1]  # drop the 1280 head
        # output stride 16: the stride-2 block at features[14] becomes stride 1 and
        # every depthwise conv from there on uses dilation 2 (padding 2)
        for i in range(14, len(feats)):
            ir: InvertedResidual = feats[i]
            dwc = ir.conv[1 if ir.expand != 1 else 0][0]
            dwc.stride = (1, 1)
            dwc.dilation = (2, 2)
            dwc.padding = (2, 2)
            ir.stride = 1
        self.features = nn.Sequential(*feats)
        self.aspp_conv = ConvBNReLU(320, 256, k=1)
        self.aspp_pool = ConvBNReLU(320, 256, k=1)
        self.project = ConvBNReLU(512, 256, k=1)
        self.classifier = nn.Conv2d(256, num_classes, 1)
        self.out_size = out_size

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

    def forward(self, x):
        h = self.features(x.permute(0, 3, 1, 2))
        a = self.aspp_conv(h)
        p = self.aspp_pool(h.mean((2, 3), keepdim=True)).expand_as(a)
        y = self.classifier(self.project(torch.cat([a, p], 1)))
        y = F.interpolate(y, size=(self.out_size, self.out_size), mode="bilinear", align_corners=True)
        return y.permute(0, 2, 3, 1)


def deeplabv3(seed: int = 0) -> DeepLabV3MobileNetV2:
    m = DeepLabV3MobileNetV2()
    m.reset_parameters(seed)
    return m.eval()


class FusedDeepLabV3(nn.Module):
    """Input [B,513,513,3] f32 NHWC.  Output [B,513,513,21] f32 (labels innermost)."""

    def __init__(self):
        super().__init__()

    @classmethod
    def from_reference(cls, m: DeepLabV3MobileNetV2, precision: str = "bf16", lowres: bool = False) -> "FusedDeepLabV3":
        self = cls()
        m = m.eval()
        self.f32 = precision == "fp32"
        self.lowres = bool(lowres)
        stem: ConvBNReLU = m.features[0]
        w, b = _fold(stem[0], stem[1])
        self.register_buffer("stem_w", w.permute(2, 3, 1, 0).contiguous())
        self.register_buffer("stem_b", b.contiguous())
        self.register_buffer("in_lut", input_lut(0.0, 255.0))  # uint8 input table (absorbable transform)
        blocks = []
        for ir in m.features[1:]:
            blk = Block(ir, precision)
            dwc = ir.conv[1 if ir.expand != 1 else 0][0]
            blk.dw.dilation = int(dwc.dilation[0])
            blocks.append(blk)
        self.blocks = nn.ModuleList(blocks)
        # stem + block 0 (fp32, uint8 frames: one stem_ir1 kernel over the 257x257 map)
        self.front = StemBlock1(self.stem_w.clone(), self.stem_b.clone(), self.blocks[0], self.f32)
        self.aspp_conv = PW(*_fold(m.aspp_conv[0], m.aspp_conv[1]), act=1, precision=precision)
        self.aspp_pool = PW(*_fold(m.aspp_pool[0], m.aspp_pool[1]), act=1, precision=precision)
        self.project = PW(*_fold(m.project[0], m.project[1]), act=1, precision=precision)
        # fp32: project split at the concat boundary (a: the 1x1 branch, p: image pooling)
        wpj, bpj = _fold(m.project[0], m.project[1])
        na = int(m.aspp_conv[0].out_channels)
        self.project_a = PW(wpj[:, :na].contiguous(), torch.zeros(wpj.shape[0]), act=1, precision=precision)
        self.project_p = PW(wpj[:, na:].contiguous(), bpj, act=0, precision=precision)
        wc = m.classifier.weight.detach().float()
        bc = m.classifier.bias.detach().float()
        n = wc.shape[0]
        n8 = (n + 7) // 8 * 8
        wp = torch.zeros(n8, wc.shape[1], 1, 1)
        wp[:n] = wc
        bp = torch.zeros(n8)
        bp[:n] = bc
        self.classifier = PW(wp, bp, act=0, out_f32=True, precision=precision)
        self.num_classes = int(n)
        self.out_size = int(m.out_size)
        return self

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        h = self.front(x, self.in_lut)
        i = 0
        for blk in self.blocks:
            if i > 0:  # (block 0 is in self.front)
                h = blk(h)
            i += 1
        if self.f32:
            return self._head_f32(h)
        a = self.aspp_conv(h)
        pooled = torch.ops.nnsx.avgpool(h)  # [B, 320]
        p = self.aspp_pool(pooled.view(pooled.shape[0], 1, 1, pooled.shape[1]))
        cat = torch.cat([a, p.expand(a.shape[0], a.shape[1], a.shape[2], p.shape[3])], 3).contiguous()
        y = self.classifier(self.project(cat))[..., : self.num_classes]
        if self.lowres:
            return y.contiguous()
        # NHWC viewed as channels-last NCHW: interpolate keeps channels-last, so the
        # final permute back is free and the decoder gets labels innermost
        y = y.permute(0, 3, 1, 2)
        y = F.interpolate(y, size=(self.out_size, self.out_size), mode="bilinear", align_corners=True)
        return y.permute(0, 2, 3, 1).contiguous()

    def _head_f32(self, h: torch.Tensor) -> torch.Tensor:
        B, hh, ww = h.shape[0], h.shape[1], h.shape[2]
        a = self.aspp_conv(h)
        pooled = torch.ops.nnsx.avgpool(h)  # [B, 320]
        p = self.aspp_pool(pooled.view(B, 1, 1, pooled.shape[1]))
        c = self.project_p(p)  # [B, 1, 1, 256] = W_p . p + b, the per-image bias
        y = torch.ops.nnsx.pw_conv_rowbias(a, self.project_a.wt, c.view(B, c.shape[3]), self.project_a.n, 1)
        logits = torch.empty((B, hh * ww, self.num_classes), dtype=torch.float32, device=h.device)
        torch.ops.nnsx.pw_conv_into(y, self.classifier.wt, self.classifier.bias, logits, 0, self.num_classes, 0)
        logits = logits.view(B, hh, ww, self.num_classes)
        if self.lowres:
            return logits
        return torch.ops.nnsx.upsample_bilinear(logits, self.out_size, self.out_size)


def fused_deeplabv3(seed: int = 0, precision: str = "bf16", lowres: bool = False) -> FusedDeepLabV3:
    return FusedDeepLabV3.from_reference(deeplabv3(seed), precision, lowres).eval()
