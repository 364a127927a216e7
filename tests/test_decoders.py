"""Decoder sub-plugins against the reference's own golden fixtures
(tests/nnstreamer_decoder_boundingbox, _image_segment, _pose).  Fixture files
are read in place from /root/reference (raw float tensors / text); tests skip
when the reference tree is not mounted.  The muxes run sync-mode=nosync: the
reference pairs the file frames through GStreamer preroll timestamps (pts 0
before PLAYING), which a running-time stamped stream does not reproduce.  Labels
are drawn with the reference's own 8x13 raster font (csrc/decoders/font.h), so the
RGBA output, swapped to the golden's BGRx byte order, must equal the golden file
byte for byte -- boxes and label glyphs alike."""
import os

import numpy as np
import pytest

REF = "/root/reference/tests"
# the bounding-box fixtures travel in-tree (tests/fixtures, copied from the reference's
# tests/nnstreamer_decoder_boundingbox) so GPU boxes without the reference run them too
_LOCAL_BB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fixtures", "nnstreamer_decoder_boundingbox")
BB = _LOCAL_BB if os.path.isdir(_LOCAL_BB) else f"{REF}/nnstreamer_decoder_boundingbox"

needs_ref = pytest.mark.skipif(not os.path.isdir(BB), reason="reference fixtures not mounted")


def _run_frames(nns, desc, n):
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes()))
    msg = p.run(timeout=60)
    p.stop()
    assert len(out) == n, (msg, p.messages())
    return out


def _rgba_to_red_mask(buf, w, h):
    a = np.frombuffer(buf, np.uint8).reshape(h, w, 4)
    return (a[..., 0] == 255) & (a[..., 1] == 0) & (a[..., 2] == 0)


def _bgrx_red_mask(path, w, h):
    a = np.fromfile(path, np.uint8).reshape(h, w, 4)
    return (a[..., 2] == 255) & (a[..., 1] == 0) & (a[..., 0] == 0)


def _compare_with_golden(mine, golden_paths, w, h):
    """Byte-exact: the decoder's RGBA frame in the golden's BGRx byte order."""
    for m, g in zip(mine, golden_paths):
        bgrx = np.frombuffer(m, np.uint8).reshape(h, w, 4)[..., [2, 1, 0, 3]]
        gold = np.fromfile(g, np.uint8).reshape(h, w, 4)
        diff = np.argwhere(np.any(bgrx != gold, axis=-1))
        assert diff.size == 0, f"{g}: {len(diff)} pixels differ, first {diff[:10].tolist()}"
        assert _bgrx_red_mask(g, w, h).any()


def _ssd_desc(mode, style, dev=-1):
    return (f"tensor_mux name=mux sync-mode=nosync ! tensor_decoder mode=bounding_boxes option1={mode} device={dev} "
            f"option2={BB}/coco_labels_list.txt option3={BB}/box_priors.txt option4=160:120 option5=300:300 "
            f"option9={style} ! tensor_sink name=sink "
            f"multifilesrc location={BB}/mobilenetssd_tensors.0.%d start-index=0 stop-index=1 "
            "caps=application/octet-stream ! tensor_converter input-dim=4:1:1917:1 input-type=float32 ! mux.sink_0 "
            f"multifilesrc location={BB}/mobilenetssd_tensors.1.%d start-index=0 stop-index=1 "
            "caps=application/octet-stream ! tensor_converter input-dim=91:1917:1 input-type=float32 ! mux.sink_1")


@needs_ref
@pytest.mark.parametrize("mode", ["mobilenet-ssd", "tflite-ssd"])
def test_bbox_mobilenet_ssd_golden(nns, mode):
    mine = _run_frames(nns, _ssd_desc(mode, "font"), 2)
    _compare_with_golden(mine, [f"{BB}/mobilenetssd_golden.{i}" for i in range(2)], 160, 120)


def _pp_desc(mode, style, dev=-1):
    src = ""
    dims = ["1", "100:1", "100:1", "4:100:1"]
    for i, d in enumerate(dims):
        src += (f" multifilesrc location={BB}/mobilenetssd_postprocess_tensors.{i}.%d start-index=0 stop-index=1 "
                f"caps=application/octet-stream ! tensor_converter input-dim={d} input-type=float32 ! mux.sink_{i}")
    return (f"tensor_mux name=mux sync-mode=nosync ! tensor_decoder mode=bounding_boxes option1={mode} device={dev} "
            f"option2={BB}/coco_labels_list.txt option4=160:120 option5=640:480 option9={style} "
            "! tensor_sink name=sink" + src)


@needs_ref
@pytest.mark.parametrize("mode", ["mobilenet-ssd-postprocess", "tf-ssd"])
def test_bbox_ssd_postprocess_golden(nns, mode):
    mine = _run_frames(nns, _pp_desc(mode, "font"), 2)
    _compare_with_golden(mine, [f"{BB}/mobilenetssd_postprocess_golden.{i}" for i in range(2)], 160, 120)


def _palm_desc(dev=-1):
    return (f"tensor_mux name=mux sync-mode=nosync ! tensor_decoder mode=bounding_boxes option1=mp-palm-detection "
            f"device={dev} "
            "option3=0.5:4:1.0:1.0:0.5:0.5:8:16:16:16 option4=160:120 option5=300:300 ! tensor_sink name=sink "
            f"multifilesrc location={BB}/palm_detection_input_0.%d start-index=0 stop-index=1 "
            "caps=application/octet-stream ! tensor_converter input-dim=18:2016:1:1 input-type=float32 ! mux.sink_0 "
            f"multifilesrc location={BB}/palm_detection_input_1.%d start-index=0 stop-index=1 "
            "caps=application/octet-stream ! tensor_converter input-dim=1:2016:1:1 input-type=float32 ! mux.sink_1")


@needs_ref
def test_bbox_palm_detection_golden(nns):
    mine = _run_frames(nns, _palm_desc(), 2)
    for i, m in enumerate(mine):
        g = np.fromfile(f"{BB}/palm_detection_result_golden.{i}", np.uint8)
        # golden is RGBA after videoconvert: identical bytes expected (no labels in palm mode)
        assert np.array_equal(np.frombuffer(m, np.uint8), g)


def test_bbox_yolov5_synthetic(nns, workdir):
    labels = f"{workdir}/yolo_labels.txt"
    with open(labels, "w") as f:
        f.write("\n".join(f"c{i}" for i in range(3)) + "\n")
    iw = ih = 64
    n = ((iw // 32) * (ih // 32) + (iw // 16) * (ih // 16) + (iw // 8) * (ih // 8)) * 3
    x = np.zeros((n, 8), np.float32)
    # two overlapping boxes (one suppressed) and one separate box
    x[0] = [0.5, 0.5, 0.25, 0.25, 0.9, 0.1, 0.9, 0.1]
    x[1] = [0.52, 0.5, 0.25, 0.25, 0.8, 0.1, 0.9, 0.1]
    x[2] = [0.2, 0.2, 0.1, 0.1, 0.9, 0.9, 0.1, 0.1]
    caps = f"other/tensors,format=static,num_tensors=1,dimensions=8:{n}:1,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_decoder mode=bounding_boxes option1=yolov5 "
                         f"option2={labels} option4=64:64 option5=64:64 option9=none ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(x.ravel(), pts=0)
    p.get_by_name("src").end_of_stream()
    p.wait(20)
    p.stop()
    mask = _rgba_to_red_mask(out[0], 64, 64)
    # box 0: x = 32 - 8 = 24, w = 16 -> columns 24..40 on rows 24 and 40
    assert mask[24, 24:41].all() and mask[40, 24:41].all()
    # box 1 (shifted by ~1 px) is suppressed: its right edge column 41 has no vertical line
    assert not mask[30, 41]
    # box 2: x = 12.8 - 3.2 = 9 -> (9, 9) .. (15, 15)
    assert mask[9, 9:16].all()


def test_bbox_batched_equals_per_frame(nns, workdir):
    from test_gpu_elements import _bbox_run, _ssd_fixture
    pri, lab, boxes, logits = _ssd_fixture(workdir, batch=3, seed=3)
    batched = _bbox_run(nns, pri, lab, boxes, logits, -1, 3)
    assert len(batched) == 3
    for i in range(3):
        single = _bbox_run(nns, pri, lab, boxes[i:i + 1], logits[i:i + 1], -1, 1)
        assert single[0][1] == batched[i][1]


# ------------------------------------------------------------ image_segment ----

def _seg_run(nns, mode, arr, dims, dev=-1, extra=""):
    caps = f"other/tensors,format=static,num_tensors=1,dimensions={dims},types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_transform mode=typecast option=float32 device={dev} "
                         f"! tensor_decoder mode=image_segment option1={mode} {extra} ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(np.frombuffer(b.memory(0).bytes(), np.uint32).copy()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(arr.ravel(), pts=0, duration=100)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(30)
    caps_out = p.get_by_name("sink").pad_caps("sink")
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    return out, caps_out


def _seg_color(label, max_labels=20):
    mod = 0xFFFFFF // (max_labels + 1)
    return 0 if label == 0 else ((mod * label) & 0xFFFFFF) | 0xFF000000


def test_image_segment_tflite_deeplab(nns):
    rng = np.random.default_rng(0)
    h, w, L = 7, 9, 21
    prob = rng.uniform(0, 0.4, (h, w, L)).astype(np.float32)
    lab = rng.integers(0, L, (h, w))
    for y in range(h):
        for x in range(w):
            if (x + y) % 3:
                prob[y, x, lab[y, x]] = 0.9   # confident pixel
    out, caps = _seg_run(nns, "tflite-deeplab", prob, f"{L}:{w}:{h}:1")
    assert caps.get("width") == w and caps.get("height") == h
    exp = np.array([_seg_color(int(lab[y, x])) if (x + y) % 3 else 0 for y in range(h) for x in range(w)], np.uint32)
    np.testing.assert_array_equal(out[0], exp)


def test_image_segment_snpe_modes(nns):
    idx = np.array([[0, 1, 2], [20, 21, -1]], np.float32)
    out, caps = _seg_run(nns, "snpe-deeplab", idx, "3:2:1")
    np.testing.assert_array_equal(out[0], [0, _seg_color(1), _seg_color(2), _seg_color(20), 0, 0])
    depth = np.array([0, 1, 2, 4], np.float32)
    out, _ = _seg_run(nns, "snpe-depth", depth, "1:2:2")
    g = [0, 63, 127, 255]
    np.testing.assert_array_equal(out[0], [v | v << 8 | v << 16 | 0xFF000000 for v in g])


def test_image_segment_batched(nns):
    rng = np.random.default_rng(1)
    prob = rng.uniform(0, 1, (3, 4, 5, 21)).astype(np.float32)
    out, _ = _seg_run(nns, "tflite-deeplab", prob, "21:5:4:3")
    assert len(out) == 3
    for b in range(3):
        single, _ = _seg_run(nns, "tflite-deeplab", prob[b], "21:5:4:1")
        np.testing.assert_array_equal(out[b], single[0])


def _seg_resized_expected(prob, W, H, thr=0.5, max_labels=20):
    """argmax of F.interpolate(bilinear, align_corners) of the label scores"""
    import torch
    t = torch.from_numpy(prob).permute(0, 3, 1, 2)
    up = torch.nn.functional.interpolate(t, size=(H, W), mode="bilinear", align_corners=True).permute(0, 2, 3, 1)
    best, idx = up.max(-1)
    col = np.vectorize(lambda l: _seg_color(int(l), max_labels), otypes=[np.uint32])(idx.numpy())
    return np.where(best.numpy() > thr, col, 0).astype(np.uint32), up.numpy()


def test_image_segment_option3_resizes_before_argmax(nns):
    """nnsx option3=W:H: a low-resolution score map is resized (bilinear,
    align_corners) per label before the argmax -- the decoded frame equals
    argmax(F.interpolate(...)) of the full-resolution scores"""
    rng = np.random.default_rng(3)
    b, h, w, L, W, H = 2, 5, 6, 21, 23, 17
    prob = rng.uniform(0, 1, (b, h, w, L)).astype(np.float32)
    out, caps = _seg_run(nns, "tflite-deeplab", prob, f"{L}:{w}:{h}:{b}", extra="option3=23:17")
    assert caps.get("width") == W and caps.get("height") == H
    exp, up = _seg_resized_expected(prob, W, H)
    for i in range(b):
        got = out[i].reshape(H, W)
        diff = got != exp[i]
        if diff.any():  # only where two labels tie to fp32 rounding (different fma order)
            s = np.sort(up[i][diff], -1)
            assert np.all(s[:, -1] - s[:, -2] < 1e-5), np.argwhere(diff)[:4]
    # same size: option3 is a no-op
    out2, caps2 = _seg_run(nns, "tflite-deeplab", prob[:1], f"{L}:{w}:{h}:1", extra=f"option3={w}:{h}")
    ref, _ = _seg_run(nns, "tflite-deeplab", prob[:1], f"{L}:{w}:{h}:1")
    assert caps2.get("width") == w
    np.testing.assert_array_equal(out2[0], ref[0])


# ---------------------------------------------------------- pose_estimation ----

def test_pose_heatmap_only(nns):
    K, gw, gh = 14, 8, 6
    heat = np.zeros((gh, gw, K), np.float32)
    peaks = {0: (1, 1), 1: (3, 2), 2: (5, 2)}
    for k, (x, y) in peaks.items():
        heat[y, x, k] = 0.9
    caps = f"other/tensors,format=static,num_tensors=1,dimensions={K}:{gw}:{gh}:1,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_decoder mode=pose_estimation option1=160:120 "
                         f"option2={gw}:{gh} ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(np.frombuffer(b.memory(0).bytes(), np.uint32).copy()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(heat.ravel(), pts=0)
    p.get_by_name("src").end_of_stream()
    p.wait(20)
    p.stop()
    img = out[0].reshape(120, 160)
    # keypoint 1 (neck) at grid (3, 2) -> pixel (60, 40); connection 0-1 drawn with an end dot
    assert img[40, 60] == 0xFFFFFFFF
    assert img[40 + 3, 60] == 0xFFFFFFFF   # end dot radius
    # midpoint of top(20,20)->neck(60,40) lies on the Bresenham line
    assert (img[29:32, 39:42] == 0xFFFFFFFF).any()
    # keypoints without a peak (score FLT_MIN < 0.5) are not drawn: bottom-right is empty
    assert (img[90:, 120:] == 0).all()


def test_pose_reference_pipelines_run(nns):
    # tests/nnstreamer_decoder_pose/runTest.sh: RGB frames split + transposed as a fake heatmap
    desc = ("videotestsrc num-buffers=4 ! video/x-raw,width=14,height=14,format=RGB ! tensor_converter "
            "! tensor_transform mode=arithmetic option=typecast:float32,add:128,div:255 "
            "! tensor_split name=a tensorseg=1:14:14:1,2:14:14:1 a.src_0 ! tensor_transform mode=transpose "
            "option=1:2:0:3 ! tensor_decoder mode=pose_estimation option1=320:240 option2=14:14 ! tensor_sink name=sink "
            "a.src_1 ! queue ! fakesink")
    p = nns.parse_launch(desc)
    n = []
    p.get_by_name("sink").connect("new-data", lambda b: n.append(b.memory(0).size))
    p.run(timeout=30)
    p.stop()
    assert n == [320 * 240 * 4] * 4
