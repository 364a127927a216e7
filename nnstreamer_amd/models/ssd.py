"""SSDLite-MobileNetV2 300x300 (COCO, 91 classes, 1917 anchors), random init.

Shapes match what the reference's bounding_boxes decoder consumes in
``mobilenet-ssd`` mode (tensordec-boundingbox.c:1006-1040 and
tests/nnstreamer_decoder_boundingbox/runTest.sh): box encodings
``4:1:1917:B`` and class logits ``91:1917:B``.  ``write_box_priors`` writes
the matching anchor file (4 lines: ycenter, xcenter, h, w) from the standard
multiple-grid SSD anchor generator.

* ``SSDLiteMobileNetV2`` -- plain Conv+BN+ReLU6 definition (fp32 oracle).
* ``FusedSSDLite``       -- BN-folded NHWC bf16 inference form on the CDNA4
  kernels (stem / depthwise / MFMA pointwise, see fused.py).
Input for both: ``[B, 300, 300, 3]`` float32 NHWC (NNStreamer ``3:300:300:B``).
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

from .fused import DW, PW, Block, StemBlock1, _fold, input_lut, stem
from .mobilenet_v2 import ConvBNReLU, MobileNetV2

ANCHORS = (3, 6, 6, 6, 6, 6)
FEATURE_SIZES = (19, 10, 5, 3, 2, 1)
NUM_ANCHORS = sum(a * s * s for a, s in zip(ANCHORS, FEATURE_SIZES))  # 1917


class SepHead(nn.Module):
    """SSDLite predictor: depthwise 3x3 + BN + ReLU6, then 1x1 conv with bias."""

    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.dw = ConvBNReLU(cin, cin, k=3, groups=cin)
        self.pw = nn.Conv2d(cin, cout, 1)

    def forward(self, x):
        return self.pw(self.dw(x))


class Extra(nn.Sequential):
    def __init__(self, cin: int, mid: int, cout: int):
        super().__init__(ConvBNReLU(cin, mid, k=1), ConvBNReLU(mid, mid, k=3, stride=2, groups=mid),
                         ConvBNReLU(mid, cout, k=1))


class SSDLiteMobileNetV2(nn.Module):
    def __init__(self, num_classes: int = 91):
        super().__init__()
        self.num_classes = num_classes
        self.features = MobileNetV2().features
        self.extras = nn.ModuleList([Extra(1280, 256, 512), Extra(512, 128, 256), Extra(256, 128, 256),
                                     Extra(256, 64, 128)])
        chans = (576, 1280, 512, 256, 256, 128)
        self.box_heads = nn.ModuleList([SepHead(c, a * 4) for c, a in zip(chans, ANCHORS)])
        self.cls_heads = nn.ModuleList([SepHead(c, a * num_classes) for c, a in zip(chans, ANCHORS)])

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
            for h in self.box_heads:
                h.pw.weight.mul_(0.05)
            for h in self.cls_heads:
                # focal-loss style prior: background dominates, a few anchors fire
                h.pw.weight.mul_(0.05)
                h.pw.bias.fill_(-math.log((1 - 0.01) / 0.01))

    def _heads(self, feats: List[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
        boxes, logits = [], []
        for f, bh, ch in zip(feats, self.box_heads, self.cls_heads):
            b = f.shape[0]
            boxes.append(bh(f).permute(0, 2, 3, 1).reshape(b, -1, 4))
            logits.append(ch(f).permute(0, 2, 3, 1).reshape(b, -1, self.num_classes))
        bx = torch.cat(boxes, 1)
        return bx.reshape(bx.shape[0], bx.shape[1], 1, 4), torch.cat(logits, 1)

    def forward(self, x):
        h = x.permute(0, 3, 1, 2)
        for i in range(14):
            h = self.features[i](h)
        blk = self.features[14]
        f1 = blk.conv[0](h)  # expansion output, 576 @ 19x19 (SSD feature 1)
        h = blk.conv[2](blk.conv[1](f1))
        for i in range(15, len(self.features)):
            h = self.features[i](h)
        feats = [f1, h]
        for e in self.extras:
            h = e(h)
            feats.append(h)
        return self._heads(feats)


def ssd_mobilenet(seed: int = 0) -> SSDLiteMobileNetV2:
    m = SSDLiteMobileNetV2()
    m.reset_parameters(seed)
    return m.eval()


def _pad_rows(w: torch.Tensor, b: torch.Tensor, mult: int = 8):
    n = w.shape[0]
    n8 = (n + mult - 1) // mult * mult
    if n8 == n:
        return w, b
    wp = torch.zeros((n8,) + tuple(w.shape[1:]), dtype=w.dtype)
    wp[:n] = w
    bp = torch.zeros(n8, dtype=b.dtype)
    bp[:n] = b
    return wp, bp


class FusedSepHead(nn.Module):
    def __init__(self, h: SepHead, k: int, precision: str = "bf16"):
        super().__init__()
        self.dw = DW(*_fold(h.dw[0], h.dw[1]), stride=1, precision=precision)
        w, b = _pad_rows(h.pw.weight.detach().float(), h.pw.bias.detach().float())
        self.pw = PW(w, b, act=0, out_f32=True, precision=precision)
        self.n = int(h.pw.out_channels)
        self.k = int(k)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.pw(self.dw(x))
        b = y.shape[0]
        if y.shape[-1] != self.n:
            y = y[..., : self.n]
        return y.reshape(b, -1, self.k)

    def into(self, x: torch.Tensor, out: torch.Tensor, row0: int) -> int:
        """fp32: the head GEMM writes its rows of the concatenated output `out`
        [B, rows, k] directly (no per-head tensor, no torch.cat).  Returns the
        next free row."""
        h = self.dw(x)
        torch.ops.nnsx.pw_conv_into(h, self.pw.wt, self.pw.bias, out, row0, self.n, 0)
        return row0 + h.shape[1] * h.shape[2] * (self.n // self.k)


class FusedExtra(nn.Module):
    def __init__(self, e: Extra, precision: str = "bf16"):
        super().__init__()
        self.a = PW(*_fold(e[0][0], e[0][1]), act=1, precision=precision)
        self.d = DW(*_fold(e[1][0], e[1][1]), stride=2, precision=precision)
        self.c = PW(*_fold(e[2][0], e[2][1]), act=1, precision=precision)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.c(self.d(self.a(x)))


class FusedSSDLite(nn.Module):
    """Input [B,300,300,3] f32 NHWC.  Outputs (boxes [B,1917,1,4] f32, logits [B,1917,91] f32)."""

    def __init__(self):
        super().__init__()

    @classmethod
    def from_reference(cls, m: SSDLiteMobileNetV2, precision: str = "bf16") -> "FusedSSDLite":
        self = cls()
        m = m.eval()
        self.f32 = precision == "fp32"
        stem: ConvBNReLU = m.features[0]
        w, b = _fold(stem[0], stem[1])
        self.register_buffer("stem_w", w.permute(2, 3, 1, 0).contiguous())
        self.register_buffer("stem_b", b.contiguous())
        self.register_buffer("in_lut", input_lut(-127.5, 127.5))  # uint8 input table (absorbable transform)
        self.blocks = nn.ModuleList([Block(ir, precision) for ir in m.features[1:-1]])  # features[1..17]
        # stem + block 0 (fp32, uint8 frames: one stem_ir1 kernel)
        self.front = StemBlock1(self.stem_w.clone(), self.stem_b.clone(), self.blocks[0], self.f32)
        head: ConvBNReLU = m.features[-1]
        self.head = PW(*_fold(head[0], head[1]), act=1, precision=precision)
        self.extras = nn.ModuleList([FusedExtra(e, precision) for e in m.extras])
        self.box_heads = nn.ModuleList([FusedSepHead(h, 4, precision) for h in m.box_heads])
        self.cls_heads = nn.ModuleList([FusedSepHead(h, m.num_classes, precision) for h in m.cls_heads])
        self.feat_block = 13  # blocks[13] == features[14]: its expansion output is SSD feature 1
        # fp32: all 12 heads (depthwise + predictor, box and class, 6 maps) through
        # nnsx::sep_heads: one grouped depthwise launch + one grouped GEMM launch
        # (the depthwise inside the GEMM's staging measured slower and was removed:
        # profiles/r4_dwpw_ab.txt)
        self.one_launch_heads = self.f32
        self.heads_mode = 0
        return self

    def forward(self, x: torch.Tensor):
        h = self.front(x, self.in_lut)
        feats: List[torch.Tensor] = []
        for i, blk in enumerate(self.blocks):
            if i == self.feat_block:
                e = blk.expand(h)
                feats.append(e)
                h = blk.project(blk.dw(e))
            elif i > 0:  # (block 0 is in self.front)
                h = blk(h)
        h = self.head(h)
        feats.append(h)
        for ex in self.extras:
            h = ex(h)
            feats.append(h)
        if self.f32 and x.is_cuda:
            rows = 0
            for i, bh in enumerate(self.box_heads):
                rows += feats[i].shape[1] * feats[i].shape[2] * (bh.n // bh.k)
            bo = torch.empty((x.shape[0], rows, 4), dtype=torch.float32, device=x.device)
            lo = torch.empty((x.shape[0], rows, self.cls_heads[0].k), dtype=torch.float32, device=x.device)
            if self.one_launch_heads:
                xs: List[torch.Tensor] = []
                wds: List[torch.Tensor] = []
                bds: List[torch.Tensor] = []
                wts: List[torch.Tensor] = []
                bs: List[torch.Tensor] = []
                ns: List[int] = []
                which: List[int] = []
                # the large maps first: their tiles start first, the small maps fill the tail
                for j, hc in enumerate(self.cls_heads):
                    xs.append(feats[j])
                    wds.append(hc.dw.w)
                    bds.append(hc.dw.bias)
                    wts.append(hc.pw.wt)
                    bs.append(hc.pw.bias)
                    ns.append(hc.n)
                    which.append(1)
                for j, hb in enumerate(self.box_heads):
                    xs.append(feats[j])
                    wds.append(hb.dw.w)
                    bds.append(hb.dw.bias)
                    wts.append(hb.pw.wt)
                    bs.append(hb.pw.bias)
                    ns.append(hb.n)
                    which.append(0)
                torch.ops.nnsx.sep_heads(xs, wds, bds, wts, bs, ns, which, bo, lo, self.heads_mode)
                return bo.reshape(bo.shape[0], bo.shape[1], 1, 4), lo
            r = 0
            for i, bh in enumerate(self.box_heads):
                r = bh.into(feats[i], bo, r)
            r = 0
            for i, ch in enumerate(self.cls_heads):
                r = ch.into(feats[i], lo, r)
            return bo.reshape(bo.shape[0], bo.shape[1], 1, 4), lo
        boxes: List[torch.Tensor] = []
        logits: List[torch.Tensor] = []
        for i, bh in enumerate(self.box_heads):
            boxes.append(bh(feats[i]))
        for i, ch in enumerate(self.cls_heads):
            logits.append(ch(feats[i]))
        bx = torch.cat(boxes, 1)
        return bx.reshape(bx.shape[0], bx.shape[1], 1, 4), torch.cat(logits, 1)


def fused_ssd_mobilenet(seed: int = 0, precision: str = "bf16") -> FusedSSDLite:
    return FusedSSDLite.from_reference(ssd_mobilenet(seed), precision).eval()


def box_priors(min_scale: float = 0.2, max_scale: float = 0.95):
    """Anchors (ycenter, xcenter, h, w) in the decoder's order: feature map,
    then location (row-major), then anchor."""
    n = len(FEATURE_SIZES)
    scales = [min_scale + (max_scale - min_scale) * i / (n - 1) for i in range(n)] + [1.0]
    rows: List[Tuple[float, float, float, float]] = []
    for li, fs in enumerate(FEATURE_SIZES):
        if li == 0:
            shapes = [(0.1, 1.0), (scales[0], 2.0), (scales[0], 0.5)]
        else:
            s = scales[li]
            shapes = [(s, 1.0), (s, 2.0), (s, 0.5), (s, 3.0), (s, 1.0 / 3.0), (math.sqrt(s * scales[li + 1]), 1.0)]
        for y in range(fs):
            for x in range(fs):
                cy, cx = (y + 0.5) / fs, (x + 0.5) / fs
                for sc, ar in shapes:
                    r = math.sqrt(ar)
                    rows.append((cy, cx, sc / r, sc * r))
    assert len(rows) == NUM_ANCHORS
    return rows


def write_box_priors(path: str) -> str:
    rows = box_priors()
    with open(path, "w") as f:
        for k in range(4):
            f.write(" ".join(f"{r[k]:.8f}" for r in rows) + "\n")
    return path


def write_coco_labels(path: str, n: int = 91) -> str:
    with open(path, "w") as f:
        f.write("\n".join(["???"] + [f"obj{i}" for i in range(1, n)]) + "\n")
    return path
