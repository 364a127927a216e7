"""A plain TorchScript MobileNetV2 (models/export.py build_model: Conv + BN +
ReLU6, NCHW inside an NHWC wrapper) loaded by tensor_filter framework=pytorch
on a GPU runs on the nnsx kernels after the load-time lowering
(csrc/filter/torch_lower.cc).  VERDICT r5 item 3: top-1 equal to torch fp32
on 512 images with max relative logit error < 1e-3; the filter reports the
lowering; an unmatched model runs unchanged.  Reference:
tensor_filter_pytorch.cc:205-230 (load), :517-557 (invoke)."""
import os

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_lowered_plain_model_matches_torch_fp32(nns, tmp_path):
    from nnstreamer_amd.models.export import export
    from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2

    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    src = export("mobilenet_v2", os.path.join(tmp_path, "plain.pt"), seed=6, layout="nhwc")
    dst = os.path.join(tmp_path, "plain_low.pt")
    rep = nns._C.lower_torchscript(src, dst, 0)
    assert "16 fused inverted residuals" in rep, rep
    low = torch.jit.load(dst, map_location="cuda").eval()
    low.in_lut.copy_(((torch.arange(256, dtype=torch.float32) - 127.5) / 127.5).cuda())
    ref = mobilenet_v2(seed=6).cuda().eval()
    g = torch.Generator().manual_seed(6)
    agree, worst = 0, 0.0
    for _ in range(2):  # 512 images, the bench batch
        x = torch.randint(0, 256, (256, 224, 224, 3), generator=g, dtype=torch.uint8).cuda()
        with torch.no_grad():
            r = ref(((x.float() - 127.5) / 127.5).permute(0, 3, 1, 2))
            y = low(x)
        agree += int((y.argmax(1) == r.argmax(1)).sum())
        worst = max(worst, ((y - r).abs().max() / r.abs().max()).item())
    assert agree == 512, agree
    assert worst < 1e-3, worst


def test_filter_lowers_plain_model_and_labels_match(nns, workdir, labels):
    from nnstreamer_amd.models.export import export
    from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2

    model = export("mobilenet_v2", os.path.join(workdir, "plain_filter.pt"), layout="nhwc")
    B, nb = 32, 4
    desc = (f"videotestsrc num-buffers={B * nb} pattern=snow pool-size=128 "
            "! video/x-raw,format=RGB,width=224,height=224,framerate=0/1 "
            f"! tee name=t t. ! queue ! tensor_converter frames-per-tensor={B} device=0 "
            "! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 ! queue max-size-buffers=2 "
            f"! tensor_filter name=f framework=pytorch model={model} input=3:224:224:{B} inputtype=float32 "
            "accelerator=true:gpu device=0 custom=hipgraph:true ! queue max-size-buffers=4 "
            f"! tensor_decoder mode=image_labeling option1={labels} ! tensor_sink name=sink "
            f"t. ! queue ! tensor_converter frames-per-tensor={B} ! appsink name=raw")
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes().decode()))
    raw = p.get_by_name("raw")
    p.set_state("playing")
    frames = []
    while len(frames) < nb:
        b = raw.pull(timeout=60)
        assert b is not None
        frames.append(b.memory(0).numpy("uint8").copy())
    p.wait(timeout=180)
    f = p.get_by_name("f")
    lowered, absorbed = f.get_property("lowered"), f.get_property("absorbed")
    p.stop()
    assert "16 fused inverted residuals" in lowered, lowered
    assert absorbed, "the transform was not absorbed into the lowered model's input table"
    assert len(out) == nb
    m = mobilenet_v2(seed=0).cuda().eval()
    agree = 0
    for txt, fr in zip(out, frames):
        x = torch.from_numpy(fr).cuda().view(B, 224, 224, 3).float()
        with torch.no_grad():
            ref = m(((x - 127.5) / 127.5).permute(0, 3, 1, 2)).argmax(1).tolist()
        agree += sum(a == f"class_{i}" for a, i in zip(txt.split("\n"), ref))
    assert agree == B * nb, agree


def test_filter_keeps_unmatched_model(nns, workdir):
    import numpy as np

    m = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 7, stride=3), torch.nn.Tanh(), torch.nn.Flatten())
    path = os.path.join(workdir, "unmatched.pt")
    torch.jit.script(m.eval()).save(path)
    p = nns.parse_launch(f"appsrc name=src caps=other/tensors,format=static,num_tensors=1,dimensions=16:16:3:1,"
                         f"types=float32,framerate=0/1 ! tensor_filter name=f framework=pytorch model={path} "
                         f"input=16:16:3:1 inputtype=float32 accelerator=true:gpu device=0 ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).numpy("float32").copy()))
    p.set_state("playing")
    x = np.random.default_rng(0).standard_normal((1, 3, 16, 16)).astype(np.float32)
    p.get_by_name("src").push_buffer(x)
    p.get_by_name("src").end_of_stream()
    p.wait(timeout=60)
    assert p.get_by_name("f").get_property("lowered") == ""
    p.stop()
    with torch.no_grad():
        ref = m(torch.from_numpy(x)).numpy().ravel()
    assert len(out) == 1 and np.allclose(out[0].ravel(), ref, atol=1e-4)
