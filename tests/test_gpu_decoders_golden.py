"""bounding_boxes decoder on the GPU (device=0: candidates, sort, NMS and the
label raster all in kernels/detect.hip) against the reference goldens, byte for
byte -- the same frames the host path reproduces (tests/test_decoders.py)."""
import numpy as np
import pytest

from test_decoders import BB, _compare_with_golden, _palm_desc, _pp_desc, _run_frames, _ssd_desc, needs_ref

pytestmark = [pytest.mark.gpu, needs_ref]


@pytest.mark.parametrize("mode", ["mobilenet-ssd", "tflite-ssd"])
def test_bbox_ssd_golden_device(nns, mode):
    mine = _run_frames(nns, _ssd_desc(mode, "font", dev=0), 2)
    _compare_with_golden(mine, [f"{BB}/mobilenetssd_golden.{i}" for i in range(2)], 160, 120)


@pytest.mark.parametrize("mode", ["mobilenet-ssd-postprocess", "tf-ssd"])
def test_bbox_ssd_postprocess_golden_device(nns, mode):
    mine = _run_frames(nns, _pp_desc(mode, "font", dev=0), 2)
    _compare_with_golden(mine, [f"{BB}/mobilenetssd_postprocess_golden.{i}" for i in range(2)], 160, 120)


def test_bbox_palm_detection_golden_device(nns):
    mine = _run_frames(nns, _palm_desc(dev=0), 2)
    for i, m in enumerate(mine):
        g = np.fromfile(f"{BB}/palm_detection_result_golden.{i}", np.uint8)
        assert np.array_equal(np.frombuffer(m, np.uint8), g)


@pytest.mark.parametrize("mode", ["ov-person-detection", "ov-face-detection"])
def test_bbox_ov_device_equals_host(nns, mode):
    rng = np.random.default_rng(7)
    rows = np.zeros((200, 7), np.float32)
    n_valid = 37
    rows[:n_valid, 0] = 0
    rows[:n_valid, 2] = rng.uniform(0.5, 1.0, n_valid)
    x0 = rng.uniform(0, 0.8, n_valid)
    y0 = rng.uniform(0, 0.8, n_valid)
    rows[:n_valid, 3], rows[:n_valid, 4] = x0, y0
    rows[:n_valid, 5] = x0 + rng.uniform(0.02, 0.2, n_valid)
    rows[:n_valid, 6] = y0 + rng.uniform(0.02, 0.2, n_valid)
    rows[n_valid, 0] = -1  # end marker: later rows are ignored
    rows[n_valid + 1:n_valid + 5] = [0, 1, 0.99, 0.1, 0.1, 0.9, 0.9]
    caps = "other/tensors,format=static,num_tensors=1,dimensions=7:200:1:1,types=float32,framerate=0/1"
    frames = {}
    for dev in (-1, 0):
        p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_decoder mode=bounding_boxes option1={mode} "
                             f"option4=320:240 option5=300:300 device={dev} ! tensor_sink name=sink")
        out = []
        p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes()))
        p.set_state("playing")
        p.get_by_name("src").push_buffer(rows.ravel(), pts=0)
        p.get_by_name("src").end_of_stream()
        assert p.wait(30)[0] == "eos", p.messages()
        p.stop()
        frames[dev] = out[0]
    a, b = np.frombuffer(frames[-1], np.uint32), np.frombuffer(frames[0], np.uint32)
    assert (a != 0).sum() > 100
    assert np.array_equal(a, b), (a != b).sum()
