"""FusedMobileNetV2: the inference form of MobileNetV2 that runs on the
hand-written CDNA4 kernels through torch.ops.nnsx.*, in one of two precisions:

* ``precision="fp32"`` (reference precision, csrc/kernels/mbv2_f32.hip): fp32
  weights, activations and accumulation; the GEMMs run on
  v_mfma_f32_16x16x4_f32.  This is what the reference computes
  (tensor_filter_pytorch.cc:517-536 runs the model on float32 tensors).
* ``precision="bf16"`` (csrc/kernels/mbv2.hip, ir_fused.hip): bf16 weights and
  activations, fp32 accumulation.

* BatchNorm folded into conv weight + bias (fold in fp64, then fp32 / bf16).
* NHWC activations end to end; the input is the NNStreamer video tensor
  `3:224:224:B` (NHWC) -- no transpose needed.
* 1x1 convs (expand / project / head / classifier) are MFMA GEMMs with
  bias + ReLU6 + residual fused in the epilogue; depthwise 3x3 and the stem are
  bandwidth kernels; global average pool is its own small kernel.

The module is TorchScript-scriptable so `tensor_filter framework=pytorch` can
load it from a .pt file (the ops resolve because the filter lives in the same
native library that registers them).
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn

from .mobilenet_v2 import ConvBNReLU, InvertedResidual, MobileNetV2

import os

# (the A/B switches of earlier rounds -- unfused blocks / stem, head GEMM + pool
# as two kernels, depthwise inside the project GEMM's staging -- are gone; their
# measurements: profiles/r4_dwpw_ab.txt, r4_fp32_layers_b512_final.txt)
FUSE_IR = True
FUSE_STEM = True
HEAD_POOL = True


def _fold(conv: nn.Conv2d, bn: nn.BatchNorm2d):
    w = conv.weight.detach().double()
    scale = bn.weight.detach().double() / torch.sqrt(bn.running_var.detach().double() + bn.eps)
    w = w * scale.view(-1, 1, 1, 1)
    b = bn.bias.detach().double() - bn.running_mean.detach().double() * scale
    return w.float(), b.float()


PRECISIONS = ("bf16", "fp32")


def _pw_weight(w: torch.Tensor, precision: str = "bf16"):
    """[N, K, 1, 1] fp32 -> zero-padded weight matrix, K contiguous:
    bf16 [ceil64(N), ceil32(K)] for the bf16 GEMMs, fp32 [ceil16(N), ceil8(K)]
    for the fp32 ones."""
    n, k = w.shape[0], w.shape[1]
    if precision == "fp32":
        npad, kpad = (n + 15) // 16 * 16, (k + 7) // 8 * 8
    else:
        npad, kpad = (n + 63) // 64 * 64, (k + 31) // 32 * 32
    out = torch.zeros(npad, kpad, dtype=torch.float32)
    out[:n, :k] = w.reshape(n, k)
    return out if precision == "fp32" else out.to(torch.bfloat16)


def x3_split(w: torch.Tensor, rows: int, cols: int) -> torch.Tensor:
    """fp32 matrix -> its split-bf16 form [3, rows, cols] bf16 (hi, mid, lo;
    zero padded): w == hi + mid + lo exactly, each part the round-to-nearest
    bf16 of the residual before it -- the kernels' F32Math::kX3 operands
    (csrc/kernels/x3.h)."""
    wp = torch.zeros(rows, cols, dtype=torch.float32)
    wp[: w.shape[0], : w.shape[1]] = w.float()
    hi = wp.to(torch.bfloat16)
    r = wp - hi.float()
    mid = r.to(torch.bfloat16)
    lo = (r - mid.float()).to(torch.bfloat16)
    return torch.stack([hi, mid, lo]).contiguous()


def input_lut(add: float, div: float) -> torch.Tensor:
    """256-entry table of a uint8 input: what `tensor_transform mode=arithmetic
    option=typecast:float32,add:<add>,div:<div>` computes for every byte value,
    in the transform's own fp32 arithmetic (bit-identical to its kernel)."""
    v = torch.arange(256, dtype=torch.float32)
    return (v + torch.tensor(add, dtype=torch.float32)) / torch.tensor(div, dtype=torch.float32)


def stem(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, lut: torch.Tensor,
         out_f32: bool = False) -> torch.Tensor:
    """3x3/2 stem from either the raw uint8 frame (mapped in-kernel through
    the 256-entry input table `lut`) or an already-normalised float32 frame."""
    if x.dtype == torch.uint8:
        return torch.ops.nnsx.stem_conv_u8(x.contiguous(), w, b, 1, lut, out_f32)
    return torch.ops.nnsx.stem_conv(x.contiguous().float(), w, b, 1, out_f32)


class PW(nn.Module):
    def __init__(self, w: torch.Tensor, b: torch.Tensor, act: int, out_f32: bool = False, precision: str = "bf16"):
        super().__init__()
        self.register_buffer("wt", _pw_weight(w, precision))
        bias = torch.zeros(self.wt.shape[0], dtype=torch.float32)
        bias[: b.numel()] = b
        self.register_buffer("bias", bias)
        self.n = int(w.shape[0])
        self.act = int(act)
        self.out_f32 = bool(out_f32)

    def forward(self, x: torch.Tensor, res: Optional[torch.Tensor] = None) -> torch.Tensor:
        return torch.ops.nnsx.pw_conv(x, self.wt, self.bias, res, self.n, self.act, self.out_f32)


class DW(nn.Module):
    def __init__(self, w: torch.Tensor, b: torch.Tensor, stride: int, dilation: int = 1, act: int = 1,
                 precision: str = "bf16"):
        super().__init__()
        c = w.shape[0]
        wdt = torch.float32 if precision == "fp32" else torch.bfloat16
        self.register_buffer("w", w.reshape(c, 9).t().contiguous().to(wdt))  # [9, C]
        self.register_buffer("bias", b.contiguous())
        self.stride = int(stride)
        self.dilation = int(dilation)
        self.act = int(act)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return torch.ops.nnsx.dw_conv(x, self.w, self.bias, self.stride, self.act, self.dilation)


class Block(nn.Module):
    def __init__(self, ir: InvertedResidual, precision: str = "bf16"):
        super().__init__()
        assert precision in PRECISIONS, precision
        layers = list(ir.conv)
        self.has_expand = ir.expand != 1
        self.f32 = precision == "fp32"
        idx = 0
        if self.has_expand:
            e: ConvBNReLU = layers[0]
            self.expand = PW(*_fold(e[0], e[1]), act=1, precision=precision)
            idx = 1
        else:
            self.expand = PW(torch.zeros(8, 8, 1, 1), torch.zeros(8), act=0, precision=precision)  # unused placeholder
        d: ConvBNReLU = layers[idx]
        self.dw = DW(*_fold(d[0], d[1]), stride=ir.stride, precision=precision)
        p: ConvBNReLU = layers[idx + 1]
        self.project = PW(*_fold(p[0], p[1]), act=0, precision=precision)
        self.use_res = bool(ir.use_res)
        # fused single-kernel path (csrc/kernels/ir_fused.hip, mbv2_f32.hip): hidden activation stays in LDS
        hid = int(d[0].out_channels)
        cin = int(ir.conv[0][0].in_channels)
        self.hid = hid
        self.cin = cin
        self.cout = int(p[0].out_channels)
        # tickets of the fp32 kernel's in-launch combine of hidden-channel parts
        # (small batches): zero here, and every launch leaves them zero again
        self.register_buffer("ir_tickets", torch.zeros(768 if self.f32 else 1, dtype=torch.int32))
        if self.f32:
            self._init_f32(cin, hid)
            return
        # (the fp32 path's split-bf16 weights; TorchScript compiles both branches)
        self.register_buffer("ir_we3", torch.zeros(1, dtype=torch.bfloat16))
        self.register_buffer("ir_wp3", torch.zeros(1, dtype=torch.bfloat16))
        # hidden width padded to the kernel's 32-channel chunk with zero weights/biases
        # (padded channels stay exactly 0 through ReLU6 and contribute nothing)
        hp = (hid + 31) // 32 * 32
        we = torch.zeros(hp, self.expand.wt.shape[1], dtype=torch.bfloat16)
        be = torch.zeros(hp)
        if self.has_expand:
            we[:hid] = self.expand.wt[:hid]
            be[:hid] = self.expand.bias[:hid]
        wd = torch.zeros(9, hp, dtype=torch.bfloat16)
        wd[:, :hid] = self.dw.w
        bd = torch.zeros(hp)
        bd[:hid] = self.dw.bias
        wp = torch.zeros(self.project.wt.shape[0], hp, dtype=torch.bfloat16)
        wp[:, :hid] = self.project.wt[:, :hid]
        self.register_buffer("ir_we", we)
        self.register_buffer("ir_be", be)
        self.register_buffer("ir_wd", wd)
        self.register_buffer("ir_bd", bd)
        self.register_buffer("ir_wp", wp)
        # measured on MI355X (scripts/bench_ir.py, batch 256): the fused kernel wins on every
        # MobileNetV2 block except the 7x7 160->960->320 one (too few tiles, 20 output tiles/lane)
        self.min_tiles = 256
        self.use_ir = (bool(torch.ops.nnsx.ir_supported(int(ir.stride), cin, hp, self.cout)) and FUSE_IR
                       and (self.has_expand or hid == hp) and self.cout < 320)

    def _init_f32(self, cin: int, hid: int):
        """fp32 fused-block operands (mbv2_f32.hip): we [hid][ceil8(cin)],
        wd [9][hid], wp [ceil16(cout)][hid]; no hidden padding (hid % 16 == 0)."""
        kin = (cin + 7) // 8 * 8
        we = torch.zeros(hid, kin)
        be = torch.zeros(hid)
        if self.has_expand:
            we[:] = self.expand.wt[:hid, :kin]
            be[:] = self.expand.bias[:hid]
        self.register_buffer("ir_we", we)
        self.register_buffer("ir_be", be)
        self.register_buffer("ir_wd", self.dw.w.clone())
        self.register_buffer("ir_bd", self.dw.bias.clone())
        self.register_buffer("ir_wp", self.project.wt[:, :hid].contiguous().clone())
        # split-bf16 forms for the x3 kernels: we3 [3, hid, ceil32(cin)], wp3 [3, ceil32(cout), hid]
        self.register_buffer("ir_we3", x3_split(we[:, :cin], hid, (cin + 31) // 32 * 32))
        self.register_buffer("ir_wp3", x3_split(self.project.wt[: self.cout, :hid], (self.cout + 31) // 32 * 32, hid))
        self.min_tiles = 0
        self.use_ir = FUSE_IR and hid % 16 == 0 and (self.has_expand or hid == cin)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.f32:
            # (dilation 2: DeepLab's output-stride-16 blocks, instantiated for 33x33 maps)
            if self.use_ir and bool(torch.ops.nnsx.ir_supported_f32(
                    self.dw.stride, x.shape[1], x.shape[2], self.cin, self.hid, self.cout, self.has_expand,
                    self.dw.dilation, x.shape[0])):
                return torch.ops.nnsx.ir_block(x, self.ir_we, self.ir_be, self.ir_wd, self.ir_bd, self.ir_wp,
                                               self.project.bias, self.dw.stride, self.cout, self.has_expand,
                                               self.use_res, self.dw.dilation, self.ir_tickets, self.ir_we3,
                                               self.ir_wp3)
            if self.use_ir and self.has_expand and bool(
                    torch.ops.nnsx.ir_expand_dw_supported_f32(self.dw.stride, x.shape[1], x.shape[2], self.cin,
                                                              self.hid, x.shape[0], self.dw.dilation)):
                # expand + depthwise in one kernel (no hidden map in HBM), project as a GEMM
                h = torch.ops.nnsx.ir_expand_dw(x, self.ir_we, self.ir_be, self.ir_wd, self.ir_bd, self.dw.stride,
                                                self.dw.dilation, self.ir_we3)
            else:
                h = self.expand(x) if self.has_expand else x
                h = self.dw(h)
            if self.use_res:
                return self.project(h, x)
            return self.project(h)
        # the fused kernel walks one 8x8 output tile per workgroup slot: with fewer
        # tiles than CUs (7x7 maps below batch 256) the unfused GEMM chain is faster
        # (scripts/bench_ir.py: 56 vs 64 us at batch 128, 94 vs 67 us at batch 256)
        ho = (x.shape[1] - 1) // self.dw.stride + 1
        tiles = x.shape[0] * ((ho + 7) // 8) * ((ho + 7) // 8)
        if self.use_ir and self.dw.dilation == 1 and tiles >= self.min_tiles:
            return torch.ops.nnsx.ir_block(x, self.ir_we, self.ir_be, self.ir_wd, self.ir_bd, self.ir_wp,
                                           self.project.bias, self.dw.stride, self.cout, self.has_expand,
                                           self.use_res)
        h = self.expand(x) if self.has_expand else x
        h = self.dw(h)
        if self.use_res:
            return self.project(h, x)
        return self.project(h)


class StemBlock1(nn.Module):
    """A MobileNetV2 backbone's 3x3/2 stem and first block (t = 1, 32 -> 16).
    fp32 on a uint8 frame: one `stem_ir1` kernel -- the 32-channel stem output
    (the largest activation of the network) never leaves LDS; otherwise the
    stem op followed by block 0.  Any frame size (partial tiles are masked)."""

    def __init__(self, stem_w: torch.Tensor, stem_b: torch.Tensor, b0: Block, f32: bool):
        super().__init__()
        self.register_buffer("stem_w", stem_w)
        self.register_buffer("stem_b", stem_b)
        self.f32 = bool(f32)
        self.fused = bool(f32 and not b0.has_expand and b0.cin == 32 and b0.cout == 16
                          and b0.dw.stride == 1 and not b0.use_res and FUSE_STEM)
        self.register_buffer("s1_wd", b0.dw.w.clone() if self.fused else torch.zeros(1))
        self.register_buffer("s1_bd", b0.dw.bias.clone() if self.fused else torch.zeros(1))
        self.register_buffer("s1_wp", b0.project.wt.clone() if self.fused else torch.zeros(1))
        self.register_buffer("s1_bp", b0.project.bias.clone() if self.fused else torch.zeros(1))
        self.b0 = b0

    def forward(self, x: torch.Tensor, lut: torch.Tensor) -> torch.Tensor:
        if self.fused and x.dtype == torch.uint8 and x.is_cuda:
            return torch.ops.nnsx.stem_ir1(x.contiguous(), self.stem_w, self.stem_b, self.s1_wd, self.s1_bd,
                                           self.s1_wp, self.s1_bp, lut)
        return self.b0(stem(x, self.stem_w, self.stem_b, lut, self.f32))


class FusedMobileNetV2(nn.Module):
    """Input: [B, H, W, 3] uint8 (raw frame, mapped through `in_lut` in the
    stem) or float32 NHWC (NNStreamer `3:W:H:B`).  Output: [B, classes] fp32
    logits.

    `in_lut` ([256] f32) is the model's uint8 input contract: by default the
    MobileNetV2 normalisation (x - 127.5) / 127.5.  tensor_filter
    framework=pytorch rewrites it at caps negotiation when it absorbs an
    upstream `tensor_transform mode=arithmetic` (the transform then passes the
    uint8 frames through), so the reference pipeline string runs the fused
    uint8 stem with the transform's exact arithmetic."""

    def __init__(self):
        super().__init__()
        self.head_pool = HEAD_POOL

    @classmethod
    def from_reference(cls, m: MobileNetV2, precision: str = "bf16") -> "FusedMobileNetV2":
        assert precision in PRECISIONS, precision
        self = cls()
        m = m.eval()
        self.f32 = precision == "fp32"
        stem: ConvBNReLU = m.features[0]
        w, b = _fold(stem[0], stem[1])  # [32, 3, 3, 3]
        self.register_buffer("stem_w", w.permute(2, 3, 1, 0).contiguous())  # [ky, kx, ci, co]
        self.register_buffer("stem_b", b.contiguous())
        self.register_buffer("in_lut", input_lut(-127.5, 127.5))
        self.blocks = nn.ModuleList([Block(ir, precision) for ir in m.features[1:-1]])
        # fp32 + uint8 frames: the stem and the first (t = 1, 32 -> 16) block run as
        # one kernel (stem_ir1), the 32-channel stem output never leaves LDS
        b0 = self.blocks[0]
        self.stem_ir1 = bool(self.f32 and not b0.has_expand and b0.cin == 32 and b0.cout == 16
                             and b0.dw.stride == 1 and not b0.use_res and FUSE_STEM)
        self.register_buffer("s1_wd", b0.dw.w.clone() if self.stem_ir1 else torch.zeros(1))
        self.register_buffer("s1_bd", b0.dw.bias.clone() if self.stem_ir1 else torch.zeros(1))
        self.register_buffer("s1_wp", b0.project.wt.clone() if self.stem_ir1 else torch.zeros(1))
        self.register_buffer("s1_bp", b0.project.bias.clone() if self.stem_ir1 else torch.zeros(1))
        head: ConvBNReLU = m.features[-1]
        self.head = PW(*_fold(head[0], head[1]), act=1, precision=precision)
        fc: nn.Linear = m.classifier[1]
        self.fc = PW(fc.weight.detach().float()[:, :, None, None], fc.bias.detach().float(), act=0, out_f32=True,
                     precision=precision)
        return self

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        start = 0
        if self.stem_ir1 and x.dtype == torch.uint8 and x.is_cuda:
            h = torch.ops.nnsx.stem_ir1(x.contiguous(), self.stem_w, self.stem_b, self.s1_wd, self.s1_bd, self.s1_wp,
                                        self.s1_bp, self.in_lut)
            start = 1
        else:
            h = stem(x, self.stem_w, self.stem_b, self.in_lut, self.f32)
        i = 0
        for blk in self.blocks:
            if i >= start:
                h = blk(h)
            i += 1
        if self.f32 and h.is_cuda and (h.shape[0] <= 8 or self.head_pool):
            # head conv + ReLU6 + global average pool in one launch (small batches:
            # a workgroup per image; larger: the tiled GEMM with a pooling epilogue)
            h = torch.ops.nnsx.pw_conv_pool(h, self.head.wt, self.head.bias, self.head.n, self.head.act)
        else:
            h = self.head(h)
            h = torch.ops.nnsx.avgpool(h)
        return self.fc(h)


def fused_mobilenet_v2(seed: int = 0, precision: str = "bf16") -> FusedMobileNetV2:
    from .mobilenet_v2 import mobilenet_v2

    return FusedMobileNetV2.from_reference(mobilenet_v2(seed=seed), precision).eval()
