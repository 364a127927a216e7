"""Model families on the host: output shapes match the decoder contracts and the
fused (BN-folded, bf16, nnsx-op) forms track the plain fp32 definitions.  The
CPU implementations of torch.ops.nnsx.* are the same reference the GPU kernel
tests compare against."""
import pytest
import torch

import nnstreamer_amd  # noqa: F401  (registers torch.ops.nnsx)
from nnstreamer_amd.models import deeplab, posenet, ssd


def _close(a, b, tol):
    # bf16 activations through 20-50 random-init layers: an all-bf16 run of the plain
    # model shows the same 5-15% relative-norm drift on the deepest heads, so the check
    # is statistical (relative norm + cosine), not elementwise
    a, b = a.float().flatten(), b.float().flatten()
    rel = ((a - b).norm() / (b.norm() + 1e-12)).item()
    cos = torch.nn.functional.cosine_similarity(a, b, 0).item()
    assert rel < tol and cos > 0.98, (rel, cos)


def test_ssd_shapes_and_fused():
    m = ssd.ssd_mobilenet(seed=1)
    x = torch.rand(2, 300, 300, 3) * 2 - 1
    with torch.no_grad():
        b, c = m(x)
        fb, fc = ssd.FusedSSDLite.from_reference(m)(x)
    assert b.shape == (2, 1917, 1, 4) and c.shape == (2, 1917, 91)
    assert fb.shape == b.shape and fc.shape == c.shape
    _close(fb, b, 0.25)
    _close(fc, c, 0.25)
    # the class prior keeps most anchors below the decoder's threshold
    assert (c > 0).float().mean() < 0.2


def test_ssd_priors(tmp_path):
    rows = ssd.box_priors()
    assert len(rows) == 1917
    p = ssd.write_box_priors(str(tmp_path / "priors.txt"))
    lines = open(p).read().strip().split("\n")
    assert len(lines) == 4 and all(len(l.split()) == 1917 for l in lines)


def test_deeplab_shapes_and_fused():
    m = deeplab.deeplabv3(seed=2)
    x = torch.rand(1, 513, 513, 3)
    with torch.no_grad():
        y = m(x)
        fy = deeplab.FusedDeepLabV3.from_reference(m)(x)
    assert y.shape == (1, 513, 513, 21) and fy.shape == y.shape
    _close(fy, y, 0.25)


def test_deeplab_fp32_head_folds_the_pooling_branch():
    """fp32 head: project(cat[a, p]) as one GEMM on a + a per-image bias, the
    classifier written into a contiguous 21-label map, the hand-written resize;
    lowres ships the 33x33 logits the decoder resizes"""
    m = deeplab.deeplabv3(seed=2)
    x = (torch.rand(2, 513, 513, 3) * 255).to(torch.uint8)
    f = deeplab.FusedDeepLabV3.from_reference(m, "fp32")
    lo = deeplab.FusedDeepLabV3.from_reference(m, "fp32", lowres=True)
    with torch.no_grad():
        y = m(x.float() / 255.0)
        fy = f(x)
        ly = lo(x)
    assert fy.shape == y.shape == (2, 513, 513, 21) and fy.is_contiguous()
    rel = ((fy - y).norm() / y.norm()).item()
    assert rel < 1e-4, rel
    assert ly.shape == (2, 33, 33, 21) and ly.is_contiguous()
    up = torch.ops.nnsx.upsample_bilinear(ly, 513, 513)
    assert torch.equal(up, fy)
    ref = torch.nn.functional.interpolate(ly.permute(0, 3, 1, 2), size=(513, 513), mode="bilinear",
                                          align_corners=True).permute(0, 2, 3, 1)
    assert torch.allclose(up, ref, rtol=1e-5, atol=1e-5)
    # the per-image bias op on its own
    a = torch.randn(2, 3, 4, 16)
    wt = torch.randn(8, 16)
    bias = torch.randn(2, 8)
    r = torch.ops.nnsx.pw_conv_rowbias(a, wt, bias, 8, 0)
    assert torch.allclose(r, a @ wt.t() + bias.view(2, 1, 1, 8), atol=1e-5)


def test_posenet_shapes_and_fused():
    m = posenet.posenet(seed=3)
    x = torch.rand(2, 257, 257, 3)
    with torch.no_grad():
        h, o = m(x)
        fh, fo = posenet.FusedPoseNet.from_reference(m)(x)
    assert h.shape == (2, 9, 9, 17) and o.shape == (2, 9, 9, 34)
    _close(fh, h, 0.25)
    _close(fo, o, 0.25)


@pytest.mark.parametrize("name", ["ssd_fused", "deeplab_fused", "posenet_fused"])
def test_fused_models_script(name):
    from nnstreamer_amd.models.export import build_model
    sm = torch.jit.script(build_model(name))
    assert sm is not None


def test_ssd_and_pose_pipelines_on_host(nns, workdir):
    import os
    from conftest import run_pipeline
    from nnstreamer_amd.models.export import export
    from nnstreamer_amd.models.posenet import write_pose_labels
    from nnstreamer_amd.models.ssd import write_box_priors, write_coco_labels
    ssd_pt = export("ssd_fused", os.path.join(workdir, "ssd_cpu.pt"))
    pri = write_box_priors(f"{workdir}/priors_cpu.txt")
    lab = write_coco_labels(f"{workdir}/coco_cpu.txt")
    desc = ("videotestsrc num-buffers=2 pattern=snow ! video/x-raw,format=RGB,width=300,height=300,framerate=30/1 "
            "! tensor_converter frames-per-tensor=2 ! tensor_transform mode=arithmetic "
            "option=typecast:float32,add:-127.5,div:127.5 "
            f"! tensor_filter framework=pytorch model={ssd_pt} input=3:300:300:2 inputtype=float32 "
            f"! tensor_decoder mode=bounding_boxes option1=mobilenet-ssd option2={lab} option3={pri} "
            "option4=160:120 option5=300:300 ! tensor_sink name=sink")
    out = run_pipeline(nns, desc, collect=lambda b: b.memory(0).size, timeout=120)
    assert out == [160 * 120 * 4] * 2
    pose_pt = export("posenet_fused", os.path.join(workdir, "pose_cpu.pt"))
    pl = write_pose_labels(f"{workdir}/pose_cpu.txt")
    desc = ("videotestsrc num-buffers=1 pattern=snow ! video/x-raw,format=RGB,width=257,height=257,framerate=30/1 "
            "! tensor_converter ! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 "
            f"! tensor_filter framework=pytorch model={pose_pt} input=3:257:257:1 inputtype=float32 "
            f"! tensor_decoder mode=pose_estimation option1=320:240 option2=257:257 option3={pl} "
            "option4=heatmap-offset ! tensor_sink name=sink")
    out = run_pipeline(nns, desc, collect=lambda b: b.memory(0).size, timeout=120)
    assert out == [320 * 240 * 4]
