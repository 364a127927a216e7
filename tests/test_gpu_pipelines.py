"""End-to-end pipelines with device-resident tensors on the MI355X."""
import numpy as np
import pytest
import torch

from conftest import run_pipeline

pytestmark = pytest.mark.gpu


def test_transform_gpu_matches_cpu(nns):
    base = ("videotestsrc num-buffers=3 pattern=snow ! video/x-raw,format=RGB,width=70,height=50,framerate=30/1 "
            "! tensor_converter device={dev} ! tensor_transform mode=arithmetic "
            "option=typecast:float32,add:-127.5,div:127.5 ! tensor_transform mode=transpose option=1:2:0:3 "
            "! tensor_sink name=sink")
    cpu = run_pipeline(nns, base.format(dev=-1), collect=lambda b: b.memory(0).numpy("float32").copy())
    gpu_bufs = run_pipeline(nns, base.format(dev=0), collect=lambda b: (b.memory(0).on_device, b.memory(0).numpy("float32").copy()))
    assert all(d for d, _ in gpu_bufs), "transform output should stay device-resident"
    for a, (_, b) in zip(cpu, gpu_bufs):
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)


def test_mobilenet_pipeline_gpu_labels_match_torch(nns, mbv2_model, labels):
    B = 4
    desc = ("videotestsrc num-buffers=8 pattern=snow ! video/x-raw,format=RGB,width=224,height=224,framerate=30/1 "
            f"! tee name=t t. ! queue ! tensor_converter frames-per-tensor={B} device=0 "
            "! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 "
            f"! tensor_filter framework=pytorch model={mbv2_model} input=3:224:224:{B} inputtype=float32 accelerator=true:gpu "
            f"! tensor_decoder mode=image_labeling option1={labels} ! tensor_sink name=sink "
            f"t. ! queue ! tensor_converter frames-per-tensor={B} ! appsink name=raw")
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes().decode()))
    raw = p.get_by_name("raw")
    p.set_state("playing")
    frames = []
    while len(frames) < 2:
        b = raw.pull(timeout=60)
        assert b is not None
        frames.append(b.memory(0).numpy("uint8").copy())
    p.wait(timeout=120)
    p.stop()
    assert len(out) == 2
    m = torch.jit.load(mbv2_model).cuda().eval()
    for labels_txt, fr in zip(out, frames):
        x = torch.from_numpy(fr).float().cuda().view(B, 224, 224, 3)
        x = (x - 127.5) / 127.5
        with torch.no_grad():
            ref = m(x).argmax(1).tolist()
        assert labels_txt.split("\n") == [f"class_{i}" for i in ref]


def test_hipgraph_filter_matches_eager(nns, mbv2_model, labels):
    res = {}
    for g in ("true", "false"):
        desc = ("videotestsrc num-buffers=6 pattern=snow ! video/x-raw,format=RGB,width=224,height=224,framerate=30/1 "
                "! tensor_converter frames-per-tensor=2 device=0 "
                "! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 "
                f"! tensor_filter framework=pytorch model={mbv2_model} input=3:224:224:2 inputtype=float32 "
                f"accelerator=true:gpu custom=hipgraph:{g} ! tensor_sink name=sink")
        res[g] = run_pipeline(nns, desc, collect=lambda b: b.memory(0).numpy("float32").copy(), timeout=120)
    assert len(res["true"]) == 3
    for a, b in zip(res["true"], res["false"]):
        np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-4)
