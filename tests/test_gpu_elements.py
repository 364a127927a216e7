"""Device-resident paths of the stream / extra elements on the MI355X:
each compares the HBM path against the host path of the same pipeline."""
import numpy as np
import pytest

from conftest import run_pipeline
from test_extra_elements import _trainer_setup

pytestmark = pytest.mark.gpu

RGB = "video/x-raw,format=RGB,width=40,height=30,framerate=30/1"


def _both(nns, desc, collect):
    cpu = run_pipeline(nns, desc.format(dev=-1), collect=collect)
    gpu = run_pipeline(nns, desc.format(dev=0), collect=collect)
    return cpu, gpu


def test_merge_and_aggregator_device(nns):
    desc = (f"videotestsrc num-buffers=4 pattern=snow ! {RGB} ! tensor_converter device={{dev}} ! m.sink_0 "
            f"videotestsrc num-buffers=4 pattern=gradient ! {RGB} ! tensor_converter device={{dev}} ! m.sink_1 "
            "tensor_merge name=m mode=linear option=1 ! tensor_aggregator frames-out=2 frames-dim=3 "
            "! tensor_sink name=sink")
    collect = lambda b: (b.memory(0).on_device, b.memory(0).numpy().copy())
    cpu, gpu = _both(nns, desc, collect)
    assert len(cpu) == len(gpu) == 2
    assert all(d for d, _ in gpu)
    for (_, a), (_, b) in zip(cpu, gpu):
        np.testing.assert_array_equal(a, b)


def test_crop_device(nns):
    raw = np.random.default_rng(1).integers(0, 255, 3 * 40 * 30, dtype=np.uint8)
    regions = np.array([2, 3, 10, 7, 30, 20, 20, 20], np.uint32)
    info = np.frombuffer(nns.meta_header(1, [4, 2], format=1) + regions.tobytes(), np.uint8)
    res = {}
    for dev in (-1, 0):
        p = nns.parse_launch(
            "appsrc name=r caps=other/tensors,format=static,num_tensors=1,dimensions=3:40:30:1,types=uint8,"
            f"framerate=0/1 ! tensor_transform mode=typecast option=uint8 device={dev} ! c.raw "
            "appsrc name=i caps=other/tensors,format=flexible,framerate=0/1 ! c.info "
            "tensor_crop name=c ! tensor_sink name=sink")
        out = []
        p.get_by_name("sink").connect("new-data", lambda b: out.append(
            [(b.memory(k).on_device, b.memory(k).bytes()) for k in range(b.n_memory)]))
        p.set_state("playing")
        p.get_by_name("r").push_buffer(raw, pts=0)
        p.get_by_name("i").push_buffer(info, pts=0)
        p.get_by_name("r").end_of_stream()
        p.get_by_name("i").end_of_stream()
        p.wait(30)
        p.stop()
        res[dev] = out[0]
    assert all(d for d, _ in res[0])
    img = raw.reshape(30, 40, 3)
    for (_, c), (_, g), (x, y, w, h) in zip(res[-1], res[0], [(2, 3, 10, 7), (30, 20, 10, 10)]):
        assert c[-w * h * 3:] == img[y:y + h, x:x + w].tobytes()
        assert g[-w * h * 3:] == c[-w * h * 3:]


def test_trainer_on_gpu(nns, workdir):
    classes, feat, ntrain, nval, epochs = 4, 16, 128, 32, 3
    cfg, centers, rng = _trainer_setup(workdir, classes, feat)
    caps = f"other/tensors,format=static,num_tensors=2,dimensions={feat}:1.1:1,types=float32.int32,framerate=0/1"
    p = nns.parse_launch(
        f"appsrc name=src caps={caps} ! tensor_trainer name=tr model-config={cfg} num-inputs=1 num-labels=1 "
        f"num-training-samples={ntrain} num-validation-samples={nval} epochs={epochs} device=0 "
        "! tensor_sink name=sink")
    stats = []
    p.get_by_name("sink").connect("new-data", lambda b: stats.append(b.memory(0).numpy("float64").copy()))
    p.set_state("playing")
    for _ in range(epochs * (ntrain + nval)):
        c = int(rng.integers(classes))
        x = centers[c] + rng.normal(size=feat).astype(np.float32)
        p.get_by_name("src").push_buffer([x.astype(np.float32), np.array([c], np.int32)], pts=0)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(120)
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    assert len(stats) == 1 + epochs
    assert stats[-1][3] >= 0.9


def _ssd_fixture(workdir, n=1917, c=91, batch=1, seed=0):
    rng = np.random.default_rng(seed)
    pri = f"{workdir}/priors_{n}.txt"
    yc, xc = rng.uniform(0, 1, n), rng.uniform(0, 1, n)
    h, w = rng.uniform(0.05, 0.4, n), rng.uniform(0.05, 0.4, n)
    with open(pri, "w") as f:
        for row in (yc, xc, h, w):
            f.write(" ".join(f"{v:.6f}" for v in row) + "\n")
    lab = f"{workdir}/ssd_labels.txt"
    with open(lab, "w") as f:
        f.write("\n".join(f"label{i}" for i in range(c)) + "\n")
    boxes = rng.normal(0, 1, (batch, n, 4)).astype(np.float32)
    logits = rng.normal(-4, 2, (batch, n, c)).astype(np.float32)
    return pri, lab, boxes, logits


def _bbox_run(nns, pri, lab, boxes, logits, dev, batch):
    n, c = boxes.shape[1], logits.shape[2]
    caps = (f"other/tensors,format=static,num_tensors=2,dimensions=4:1:{n}:{batch}.{c}:{n}:{batch},"
            "types=float32.float32,framerate=0/1")
    p = nns.parse_launch(
        f"appsrc name=src caps={caps} ! tensor_transform mode=typecast option=float32 device={dev} "
        f"! tensor_decoder mode=bounding_boxes option1=mobilenet-ssd option2={lab} option3={pri} "
        "option4=320:240 option5=300:300 ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append((b.memory(0).on_device, b.memory(0).bytes())))
    p.set_state("playing")
    p.get_by_name("src").push_buffer([boxes.ravel(), logits.ravel()], pts=0, duration=4 * 33000000)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(60)
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    return out


def test_bbox_ssd_device_matches_host(nns, workdir):
    pri, lab, boxes, logits = _ssd_fixture(workdir, batch=4)
    host = _bbox_run(nns, pri, lab, boxes, logits, -1, 4)
    dev = _bbox_run(nns, pri, lab, boxes, logits, 0, 4)
    assert len(host) == len(dev) == 4
    assert all(d for d, _ in dev)
    for (_, h), (_, d) in zip(host, dev):
        a = np.frombuffer(h, np.uint32)
        b = np.frombuffer(d, np.uint32)
        assert (a != 0).sum() > 100
        # exp as fp64-rounded-once, no contraction: device frames equal the host's exactly
        assert np.array_equal(a, b), (a != b).sum()


def test_segment_device_matches_host(nns):
    from test_decoders import _seg_run
    rng = np.random.default_rng(5)
    prob = rng.uniform(0, 1, (2, 65, 67, 21)).astype(np.float32)  # odd sizes: partial LDS tiles
    host, _ = _seg_run(nns, "tflite-deeplab", prob, "21:67:65:2", dev=-1)
    dev, _ = _seg_run(nns, "tflite-deeplab", prob, "21:67:65:2", dev=0)
    for a, b in zip(host, dev):
        np.testing.assert_array_equal(a, b)
    depth = rng.uniform(0, 5, (3, 16, 16)).astype(np.float32)
    host, _ = _seg_run(nns, "snpe-depth", depth, "1:16:16:3", dev=-1)
    dev, _ = _seg_run(nns, "snpe-depth", depth, "1:16:16:3", dev=0)
    for a, b in zip(host, dev):
        np.testing.assert_array_equal(a, b)


def test_segment_resize_device_matches_host(nns):
    """option3: the fused resize + argmax + colour kernel against the host
    decoder and argmax(F.interpolate) (ties within fp32 rounding excepted)"""
    from test_decoders import _seg_resized_expected, _seg_run
    rng = np.random.default_rng(6)
    prob = rng.uniform(0, 1, (3, 33, 33, 21)).astype(np.float32)
    host, caps = _seg_run(nns, "tflite-deeplab", prob, "21:33:33:3", dev=-1, extra="option3=513:513")
    dev, _ = _seg_run(nns, "tflite-deeplab", prob, "21:33:33:3", dev=0, extra="option3=513:513")
    assert caps.get("width") == 513 and len(dev) == 3
    exp, up = _seg_resized_expected(prob, 513, 513)
    for i, (a, b) in enumerate(zip(host, dev)):
        for got in (a, b):
            diff = got.reshape(513, 513) != exp[i]
            if diff.any():
                srt = np.sort(up[i][diff], -1)
                assert np.all(srt[:, -1] - srt[:, -2] < 1e-5), np.argwhere(diff)[:4]
        assert (a != b).mean() < 1e-4


def test_pose_device_matches_host(nns):
    rng = np.random.default_rng(7)
    K, gw, gh, B = 14, 33, 33, 2
    heat = rng.uniform(-1, 1, (B, gh, gw, K)).astype(np.float32)
    res = {}
    for dev in (-1, 0):
        caps = f"other/tensors,format=static,num_tensors=1,dimensions={K}:{gw}:{gh}:{B},types=float32,framerate=0/1"
        p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_transform mode=typecast option=float32 "
                             f"device={dev} ! tensor_decoder mode=pose_estimation option1=320:240 option2=257:257 "
                             "! tensor_sink name=sink")
        out = []
        p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes()))
        p.set_state("playing")
        p.get_by_name("src").push_buffer(heat.ravel(), pts=0, duration=66)
        p.get_by_name("src").end_of_stream()
        p.wait(30)
        p.stop()
        res[dev] = out
    assert len(res[0]) == B and res[0] == res[-1]


@pytest.mark.parametrize("w,h,n,pool", [(224, 224, 6, 5), (5, 3, 7, 5), (64, 48, 130, 5), (257, 257, 9, 5),
                                         (513, 11, 3, 5), (2731, 5, 2, 5), (513, 513, 8, 64), (257, 257, 64, 128),
                                         (513, 513, 8, 3), (7, 5, 16, 40), (513, 513, 1, 5), (257, 257, 1, 5),
                                         (5, 3, 1, 5), (513, 513, 8, 12), (257, 257, 16, 20)])
def test_converter_batched_gather_matches_host(nns, w, h, n, pool):
    """Batched upload (frames-per-tensor) equals the host path byte for byte.
    Padded rows (W*3 % 4 != 0) take the DMA + unpad_rows path: one DMA over a
    run of equally spaced pool frames (a batch that wraps around the pool is
    two runs: pool 12 / batch 8, pool 20 / batch 16) or one per frame -- at
    batch 1 too (it replaced a per-row 2D copy)."""
    desc = (f"videotestsrc num-buffers={2 * n} pattern=snow pool-size={pool} ! video/x-raw,format=RGB,width={w},height={h},"
            f"framerate=30/1 ! tensor_converter frames-per-tensor={n} device={{dev}} ! tensor_sink name=sink")
    collect = lambda b: (b.memory(0).on_device, b.memory(0).bytes())
    cpu, gpu = _both(nns, desc, collect)
    assert len(cpu) == len(gpu) == 2
    assert all(d for d, _ in gpu)
    for (_, a), (_, b) in zip(cpu, gpu):
        assert a == b
