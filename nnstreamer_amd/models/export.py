"""Export random-init model families as TorchScript files for
`tensor_filter framework=pytorch model=<file>.pt` (no checkpoints or
datasets are available offline; weights are seeded random init).

    python -m nnstreamer_amd.models.export mobilenet_v2 /tmp/mbv2.pt
"""
from __future__ import annotations

import argparse
import os

import torch

from .mobilenet_v2 import mobilenet_v2


class NCHWWrapper(torch.nn.Module):
    """Accepts the NNStreamer-ordered float tensor as the pytorch filter builds
    it (dims reversed: [N, C, H, W] for `224:224:3:N`)."""

    def __init__(self, model: torch.nn.Module):
        super().__init__()
        self.model = model

    def forward(self, x):
        return self.model(x)


class NHWCWrapper(torch.nn.Module):
    """Accepts `3:W:H:N` (NNStreamer video order == NHWC) float input."""

    def __init__(self, model: torch.nn.Module):
        super().__init__()
        self.model = model

    def forward(self, x):
        return self.model(x.permute(0, 3, 1, 2))


def build_model(name: str, seed: int = 0, layout: str = "nchw", num_classes: int = 1000):
    name = name.lower().replace("-", "_")
    if name in ("mobilenet_v2", "mbv2"):
        m = mobilenet_v2(num_classes=num_classes, seed=seed)
    elif name in ("mobilenet_v2_fused", "mbv2_fused", "mobilenet_v2_fused_bf16"):
        from .fused import FusedMobileNetV2

        return FusedMobileNetV2.from_reference(mobilenet_v2(num_classes=num_classes, seed=seed)).eval()
    elif name in ("mobilenet_v2_fused_fp32", "mbv2_fused_fp32"):
        from .fused import FusedMobileNetV2

        return FusedMobileNetV2.from_reference(mobilenet_v2(num_classes=num_classes, seed=seed), "fp32").eval()
    elif name in ("ssd_mobilenet", "ssd"):
        from .ssd import ssd_mobilenet

        return ssd_mobilenet(seed=seed).eval()
    elif name in ("ssd_mobilenet_fused", "ssd_fused", "ssd_fused_fp32"):
        from .ssd import fused_ssd_mobilenet

        return fused_ssd_mobilenet(seed=seed, precision="fp32" if name.endswith("_fp32") else "bf16")
    elif name in ("deeplabv3", "deeplab"):
        from .deeplab import deeplabv3

        return deeplabv3(seed=seed).eval()
    elif name in ("deeplabv3_fused", "deeplab_fused", "deeplab_fused_fp32", "deeplab_fused_lowres",
                  "deeplab_fused_lowres_fp32"):
        from .deeplab import fused_deeplabv3

        # _lowres: 33x33 logits out; the image_segment decoder resizes (option3=513:513)
        return fused_deeplabv3(seed=seed, precision="fp32" if name.endswith("_fp32") else "bf16",
                               lowres="_lowres" in name)
    elif name in ("posenet", "pose"):
        from .posenet import posenet

        return posenet(seed=seed).eval()
    elif name in ("posenet_fused", "pose_fused", "posenet_fused_fp32"):
        from .posenet import fused_posenet

        return fused_posenet(seed=seed, precision="fp32" if name.endswith("_fp32") else "bf16")
    else:
        raise ValueError(f"unknown model {name}")
    return (NHWCWrapper(m) if layout == "nhwc" else NCHWWrapper(m)).eval()


def export(name: str, path: str, seed: int = 0, layout: str = "nchw", example_shape=None, trace: bool = False) -> str:
    model = build_model(name, seed=seed, layout=layout)
    with torch.no_grad():
        if trace:
            shape = example_shape or ((1, 3, 224, 224) if layout == "nchw" else (1, 224, 224, 3))
            sm = torch.jit.trace(model, torch.zeros(shape))
        else:
            sm = torch.jit.script(model)
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    sm.save(path)
    return path


def write_labels(path: str, n: int = 1000) -> str:
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        for i in range(n):
            f.write(f"class_{i}\n")
    return path


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("model")
    ap.add_argument("path")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--layout", default="nchw", choices=["nchw", "nhwc"])
    ap.add_argument("--trace", action="store_true")
    a = ap.parse_args()
    print(export(a.model, a.path, a.seed, a.layout, trace=a.trace))


if __name__ == "__main__":
    main()
