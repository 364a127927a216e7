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


# ------------------------------------------- BASELINE configs 3-5 on one GPU ----

def _export(workdir, name):
    import os
    from nnstreamer_amd.models.export import export
    path = os.path.join(workdir, f"{name}.pt")
    if not os.path.exists(path):
        export(name, path)
    return path


def test_ssd_pipeline_device_decoder_matches_host(nns, workdir):
    from nnstreamer_amd.models.ssd import write_box_priors, write_coco_labels
    model = _export(workdir, "ssd_fused")
    pri = write_box_priors(f"{workdir}/ssd_priors.txt")
    lab = write_coco_labels(f"{workdir}/coco.txt")
    res = {}
    for ddev in (0, -1):
        desc = ("videotestsrc num-buffers=8 pattern=snow ! video/x-raw,format=RGB,width=300,height=300,framerate=30/1 "
                "! tensor_converter frames-per-tensor=4 device=0 "
                "! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 "
                f"! tensor_filter framework=pytorch model={model} input=3:300:300:4 inputtype=float32 "
                "accelerator=true:gpu custom=hipgraph:true "
                f"! tensor_decoder mode=bounding_boxes device={ddev} option1=mobilenet-ssd option2={lab} "
                f"option3={pri} option4=320:240 option5=300:300 ! tensor_sink name=sink")
        res[ddev] = run_pipeline(nns, desc, collect=lambda b: (b.memory(0).on_device, b.memory(0).bytes()), timeout=180)
    assert len(res[0]) == len(res[-1]) == 8
    assert all(d for d, _ in res[0]) and not any(d for d, _ in res[-1])
    for (_, a), (_, b) in zip(res[0], res[-1]):
        a = np.frombuffer(a, np.uint32)
        b = np.frombuffer(b, np.uint32)
        assert np.array_equal(a, b), (a != b).sum()


def test_deeplab_pipeline(nns, workdir):
    model = _export(workdir, "deeplab_fused")
    desc = ("videotestsrc num-buffers=4 pattern=snow ! video/x-raw,format=RGB,width=513,height=513,framerate=30/1 "
            "! tensor_converter frames-per-tensor=2 device=0 "
            "! tensor_transform mode=arithmetic option=typecast:float32,div:255.0 "
            f"! tensor_filter framework=pytorch model={model} input=3:513:513:2 inputtype=float32 "
            "accelerator=true:gpu custom=hipgraph:true "
            "! tensor_decoder mode=image_segment option1=tflite-deeplab ! tensor_sink name=sink")
    out = run_pipeline(nns, desc, collect=lambda b: (b.memory(0).on_device, b.memory(0).size), timeout=180)
    assert len(out) == 4 and all(d and s == 513 * 513 * 4 for d, s in out)


def test_posenet_pipeline(nns, workdir):
    from nnstreamer_amd.models.posenet import write_pose_labels
    model = _export(workdir, "posenet_fused")
    lab = write_pose_labels(f"{workdir}/pose17.txt")
    desc = ("videotestsrc num-buffers=4 pattern=snow ! video/x-raw,format=RGB,width=257,height=257,framerate=30/1 "
            "! tensor_converter frames-per-tensor=2 device=0 "
            "! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 "
            f"! tensor_filter framework=pytorch model={model} input=3:257:257:2 inputtype=float32 "
            "accelerator=true:gpu custom=hipgraph:true "
            f"! tensor_decoder mode=pose_estimation option1=640:480 option2=257:257 option3={lab} "
            "option4=heatmap-offset ! tensor_sink name=sink")
    out = run_pipeline(nns, desc, collect=lambda b: b.memory(0).size, timeout=180)
    assert out == [640 * 480 * 4] * 4
