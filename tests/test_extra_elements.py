"""tensor_if / tensor_rate / tensor_repo / sparse / debug / join / datarepo on
the host path (reference: tests/nnstreamer_if/runTest.sh, nnstreamer_rate,
nnstreamer_repo*, nnstreamer_sparse, tests/nnstreamer_datarepo)."""
import json

import numpy as np
import pytest

from test_elements_cpu import appsrc_pipeline

U8 = "other/tensors,format=static,num_tensors=1,dimensions=4,types=uint8,framerate=0/1"
F32 = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"


def _if_run(nns, props, frames, caps=U8, two_sinks=True):
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_if name=tif {props} "
                         "tif.src_0 ! queue ! tensor_sink name=t tif.src_1 ! queue ! tensor_sink name=f")
    got = {"t": [], "f": []}
    for k in got:
        p.get_by_name(k).connect("new-data", lambda b, k=k: got[k].append([b.memory(i).numpy().copy()
                                                                          for i in range(b.n_memory)]))
    p.set_state("playing")
    for i, fr in enumerate(frames):
        p.get_by_name("src").push_buffer(fr, pts=i)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(20)
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    return got


@pytest.mark.parametrize("op,sv,expect", [
    ("EQ", "5", [False, True, False]), ("NE", "5", [True, False, True]), ("GT", "5", [False, False, True]),
    ("GE", "5", [False, True, True]), ("LT", "5", [True, False, False]), ("LE", "5", [True, True, False]),
    ("RANGE_INCLUSIVE", "4,5", [True, True, False]), ("RANGE_EXCLUSIVE", "3,6", [True, True, False]),
    ("NOT_IN_RANGE_INCLUSIVE", "5,9", [True, False, False]), ("NOT_IN_RANGE_EXCLUSIVE", "4,9", [True, False, True]),
])
def test_if_a_value_operators(nns, op, sv, expect):
    frames = [np.array([0, 0, v, 0], np.uint8) for v in (4, 5, 9)]
    got = _if_run(nns, f"compared-value=A_VALUE compared-value-option=2:0:0:0,0 supplied-value={sv} operator={op} "
                       "then=PASSTHROUGH else=PASSTHROUGH", frames)
    assert len(got["t"]) == sum(expect) and len(got["f"]) == len(expect) - sum(expect)
    tvals = [int(b[0][2]) for b in got["t"]]
    assert tvals == [v for v, e in zip((4, 5, 9), expect) if e]


def test_if_average_and_skip(nns):
    frames = [np.array([1, 2, 3, 4], np.float32), np.array([10, 10, 10, 10], np.float32)]
    got = _if_run(nns, "compared-value=TENSOR_AVERAGE_VALUE compared-value-option=0 supplied-value=5 operator=GT "
                       "then=PASSTHROUGH else=SKIP", frames, caps=F32)
    assert len(got["t"]) == 1 and len(got["f"]) == 0
    np.testing.assert_array_equal(got["t"][0][0].view(np.float32), frames[1])


def test_if_tensorpick(nns):
    caps = "other/tensors,format=static,num_tensors=3,dimensions=2.2.2,types=uint8.uint8.uint8,framerate=0/1"
    frames = [[np.array([k, k], np.uint8) for k in (1, 2, 3)]]
    got = _if_run(nns, "compared-value=A_VALUE compared-value-option=0,1 supplied-value=2 operator=EQ "
                       "then=TENSORPICK then-option=2,0 else=SKIP", frames, caps=caps)
    assert len(got["t"]) == 1
    assert [int(x[0]) for x in got["t"][0]] == [3, 1]


def test_if_custom(nns):
    nns.register_if_custom("first_is_odd", lambda arrs: bool(arrs[0].ravel()[0] % 2))
    frames = [np.array([k, 0, 0, 0], np.uint8) for k in range(4)]
    got = _if_run(nns, "compared-value=CUSTOM compared-value-option=first_is_odd then=PASSTHROUGH else=PASSTHROUGH",
                  frames)
    nns.unregister_if_custom("first_is_odd")
    assert [int(b[0][0]) for b in got["t"]] == [1, 3]
    assert [int(b[0][0]) for b in got["f"]] == [0, 2]


def test_rate_downsample_and_props(nns):
    caps = "other/tensors,format=static,num_tensors=1,dimensions=1,types=uint8,framerate=30/1"
    frames = [np.array([i], np.uint8) for i in range(30)]
    pts = [i * 1000000000 // 30 for i in range(30)]
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_rate name=r framerate=10/1 throttle=false "
                         "! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append((b.pts, int(b.memory(0).numpy()[0]))))
    p.set_state("playing")
    for f, t in zip(frames, pts):
        p.get_by_name("src").push_buffer(f, pts=t)
    p.get_by_name("src").end_of_stream()
    p.wait(20)
    r = p.get_by_name("r")
    stats = {k: int(r.get_property(k)) for k in ("in", "out", "drop", "duplicate")}
    caps_out = p.get_by_name("sink").pad_caps("sink")
    p.stop()
    # videorate selection: the held frame closest to each 100 ms slot, the last frame flushed at EOS
    assert [t for t, _ in out] == [i * 100000000 for i in range(11)]
    assert [v for _, v in out] == [3 * i for i in range(10)] + [29]
    assert stats["in"] == 30 and stats["out"] == 11 and stats["drop"] == 19 and stats["duplicate"] == 0
    assert caps_out.get("framerate") == (10, 1)


def test_rate_upsample_duplicates(nns):
    caps = "other/tensors,format=static,num_tensors=1,dimensions=1,types=uint8,framerate=5/1"
    frames = [np.array([i], np.uint8) for i in range(3)]
    out = appsrc_pipeline(nns, "tensor_rate framerate=10/1 throttle=false ! tensor_sink name=sink", caps, frames,
                          pts=[0, 200000000, 400000000])
    assert len(out) == 5
    assert [int(b.memory(0).numpy()[0]) for b in out] == [0, 0, 1, 1, 2]


def test_repo_loop_recurrence(nns):
    # accumulator: out = in + state, state fed back through tensor_repo slot 3
    caps = "other/tensors,format=static,num_tensors=1,dimensions=1,types=float32,framerate=0/1"
    nns.register_custom_easy("acc_add", lambda x: [(x[0] + x[1]).astype(np.float32)],
                             [nns.TensorShape([1], np.float32), nns.TensorShape([1], np.float32)],
                             [nns.TensorShape([1], np.float32)])
    p = nns.parse_launch(
        f"appsrc name=src caps={caps} ! mux.sink_0 "
        f"tensor_reposrc slot-index=3 caps={caps} ! mux.sink_1 "
        "tensor_mux name=mux sync-mode=nosync ! tensor_filter framework=custom-easy model=acc_add ! tee name=t "
        "t. ! queue ! tensor_reposink slot-index=3 t. ! queue ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(float(b.memory(0).numpy("float32")[0])))
    p.set_state("playing")
    for i in range(1, 6):
        p.get_by_name("src").push_buffer(np.array([i], np.float32), pts=i)
    import time
    t0 = time.time()
    while len(out) < 5 and time.time() - t0 < 20:
        time.sleep(0.01)
    p.stop()
    nns.unregister_custom_easy("acc_add")
    assert out[:5] == [1.0, 3.0, 6.0, 10.0, 15.0]


def test_sparse_roundtrip(nns):
    x = np.zeros(64, np.float32)
    x[[3, 17, 40]] = [1.5, -2.0, 7.0]
    caps = "other/tensors,format=static,num_tensors=1,dimensions=8:8,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_sparse_enc ! tee name=t "
                         "t. ! queue ! tensor_sink name=enc t. ! queue ! tensor_sparse_dec ! tensor_sink name=sink")
    enc, dec = [], []
    p.get_by_name("enc").connect("new-data", lambda b: enc.append(b.memory(0).bytes()))
    p.get_by_name("sink").connect("new-data", lambda b: dec.append(b.memory(0).numpy("float32").copy()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(x, pts=0)
    p.get_by_name("src").end_of_stream()
    p.wait(20)
    caps_out = p.get_by_name("sink").pad_caps("sink")
    p.stop()
    h = nns.parse_meta_header(enc[0][:128])
    assert h["valid"] and h["nnz"] == 3 and len(enc[0]) == 128 + 3 * 8
    np.testing.assert_array_equal(dec[0], x)
    assert caps_out.get("format") == "static"


def test_debug_passthrough(nns):
    out = appsrc_pipeline(nns, "tensor_debug output-method=console-info capability=always metadata=timestamps "
                               "! tensor_sink name=sink", U8, [np.arange(4, dtype=np.uint8)])
    np.testing.assert_array_equal(out[0].memory(0).numpy(), np.arange(4))


def test_join(nns):
    desc = (f"appsrc name=a caps={U8} ! j.sink_0 appsrc name=b caps={U8} ! j.sink_1 "
            "join name=j ! tensor_sink name=sink")
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(int(b.memory(0).numpy()[0])))
    assert p.get_by_name("j").get_property("n-pads") == "2"  # gstjoin.c:448, read-only
    p.set_state("playing")
    p.get_by_name("a").push_buffer(np.full(4, 1, np.uint8), pts=0)
    p.get_by_name("b").push_buffer(np.full(4, 2, np.uint8), pts=1)
    p.get_by_name("a").end_of_stream()
    p.get_by_name("b").end_of_stream()
    msg = p.wait(20)
    p.stop()
    assert msg and msg[0] == "eos"
    assert sorted(out) == [1, 2]


def test_datarepo_write_read_shuffle(nns, workdir):
    data = f"{workdir}/repo.dat"
    js = f"{workdir}/repo.json"
    caps = "other/tensors,format=static,num_tensors=2,dimensions=3.1,types=uint8.float32,framerate=0/1"
    frames = [[np.full(3, i, np.uint8), np.array([i * 0.5], np.float32)] for i in range(6)]
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! datareposink location={data} json={js}")
    p.set_state("playing")
    for i, f in enumerate(frames):
        p.get_by_name("src").push_buffer(f, pts=i)
    p.get_by_name("src").end_of_stream()
    assert p.wait(20)[0] == "eos"
    p.stop()
    meta = json.load(open(js))
    assert meta["total_samples"] == 6 and meta["sample_size"] == 7

    p = nns.parse_launch(f"datareposrc location={data} json={js} start-sample-index=1 stop-sample-index=4 epochs=2 "
                         "is-shuffle=true ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append((int(b.memory(0).numpy()[0]),
                                                                    float(b.memory(1).numpy("float32")[0]))))
    p.run(timeout=20)
    p.stop()
    assert len(out) == 8
    assert sorted(out[:4]) == [(i, i * 0.5) for i in range(1, 5)]
    assert sorted(out[4:]) == sorted(out[:4])


def _trainer_setup(workdir, classes=4, feat=16):
    import torch

    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(feat, 32), torch.nn.ReLU(), torch.nn.Linear(32, classes))
    path = f"{workdir}/mlp_train.pt"
    torch.jit.script(net).save(path)
    cfg = f"{workdir}/mlp_train.ini"
    with open(cfg, "w") as f:
        f.write(f"[model]\nmodel = {path}\nloss = cross_entropy\noptimizer = adam\nlearning_rate = 0.02\n"
                "batch_size = 16\n")
    rng = np.random.default_rng(0)
    centers = rng.normal(size=(classes, feat)).astype(np.float32) * 3
    return cfg, centers, rng


def test_trainer_pytorch_learns(nns, workdir):
    classes, feat, ntrain, nval, epochs = 4, 16, 128, 32, 4
    cfg, centers, rng = _trainer_setup(workdir, classes, feat)
    save = f"{workdir}/mlp_trained.pt"
    caps = (f"other/tensors,format=static,num_tensors=2,dimensions={feat}:1.1:1,types=float32.int32,"
            "framerate=0/1")
    p = nns.parse_launch(
        f"appsrc name=src caps={caps} ! tensor_trainer name=tr framework=pytorch model-config={cfg} "
        f"model-save-path={save} num-inputs=1 num-labels=1 num-training-samples={ntrain} "
        f"num-validation-samples={nval} epochs={epochs} input-dim={feat}:1,1:1 input-type=float32,int32 "
        "! tensor_sink name=sink")
    stats = []
    p.get_by_name("sink").connect("new-data", lambda b: stats.append(b.memory(0).numpy("float64").copy()))
    p.set_state("playing")
    for e in range(epochs):
        for i in range(ntrain + nval):
            c = int(rng.integers(classes))
            x = centers[c] + rng.normal(size=feat).astype(np.float32)
            p.get_by_name("src").push_buffer([x.astype(np.float32), np.array([c], np.int32)], pts=i)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(120)
    assert msg and msg[0] == "eos", p.messages()
    tr = p.get_by_name("tr")
    assert int(tr.get_property("epoch-count")) == epochs
    p.stop()
    assert len(stats) == 1 + epochs
    assert all(s.shape == (4,) for s in stats)
    first, last = stats[1], stats[-1]
    assert last[0] < first[0]                  # training loss decreases
    assert last[3] >= 0.9                      # validation accuracy on separable clusters
    import os
    assert os.path.exists(save)


def test_trainer_bad_config(nns, workdir):
    caps = "other/tensors,format=static,num_tensors=2,dimensions=4.1,types=float32.int32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_trainer model-config={workdir}/missing.ini "
                         "num-inputs=1 num-labels=1 ! tensor_sink name=sink")
    p.set_state("playing")
    p.get_by_name("src").push_buffer([np.zeros(4, np.float32), np.zeros(1, np.int32)], pts=0)
    msg = p.wait(20)
    p.stop()
    assert msg and msg[0] == "error"


def test_crop_regions(nns):
    raw = np.arange(3 * 8 * 6, dtype=np.uint8)  # [h=6][w=8][ch=3]
    regions = np.array([1, 2, 3, 2, 6, 4, 5, 5], np.uint32)  # second region clamps to the edge
    info = nns.meta_header(1, [4, 2], format=1) + regions.tobytes()  # type 1 = uint32
    p = nns.parse_launch(
        "appsrc name=r caps=other/tensors,format=static,num_tensors=1,dimensions=3:8:6:1,types=uint8,framerate=0/1 "
        "! c.raw appsrc name=i caps=other/tensors,format=flexible,framerate=0/1 ! c.info "
        "tensor_crop name=c lateness=-1 ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append([b.memory(k).bytes() for k in range(b.n_memory)]))
    p.set_state("playing")
    p.get_by_name("r").push_buffer(raw, pts=0)
    p.get_by_name("i").push_buffer(np.frombuffer(info, np.uint8), pts=0)
    p.get_by_name("r").end_of_stream()
    p.get_by_name("i").end_of_stream()
    msg = p.wait(20)
    caps = p.get_by_name("sink").pad_caps("sink")
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    assert caps.get("format") == "flexible"
    img = raw.reshape(6, 8, 3)
    assert len(out) == 1 and len(out[0]) == 2
    for blob, (x, y, w, h) in zip(out[0], [(1, 2, 3, 2), (6, 4, 2, 2)]):
        hdr = nns.parse_meta_header(blob[:128])
        assert hdr["valid"] and hdr["dims"][:3] == [3, w, h]
        np.testing.assert_array_equal(np.frombuffer(blob[128:], np.uint8), img[y:y + h, x:x + w].ravel())


def _fake_iio(root, data):
    """Fake /sys/bus/iio/devices tree + /dev node (reference tests/nnstreamer_source/unittest_src_iio.cc
    builds the same kind of tree)."""
    import os
    dev = os.path.join(root, "sys", "iio:device0")
    os.makedirs(os.path.join(dev, "scan_elements"))
    os.makedirs(os.path.join(dev, "buffer"))
    os.makedirs(os.path.join(root, "dev"))
    files = {
        "name": "fake_accel", "sampling_frequency": "1000", "in_accel_scale": "0.5", "in_accel_offset": "1",
        "buffer/length": "1", "buffer/enable": "0",
        "scan_elements/in_accel_x_en": "0", "scan_elements/in_accel_x_index": "0",
        "scan_elements/in_accel_x_type": "le:s12/16>>4",
        "scan_elements/in_accel_y_en": "0", "scan_elements/in_accel_y_index": "1",
        "scan_elements/in_accel_y_type": "be:u8/8>>0",
        "scan_elements/in_timestamp_en": "0", "scan_elements/in_timestamp_index": "2",
        "scan_elements/in_timestamp_type": "le:s64/64>>0",
    }
    for k, v in files.items():
        with open(os.path.join(dev, k), "w") as f:
            f.write(v)
    with open(os.path.join(root, "dev", "iio:device0"), "wb") as f:
        f.write(data)
    return os.path.join(root, "sys"), os.path.join(root, "dev"), dev


def test_src_iio_buffered(nns, tmp_path):
    import struct
    # scan of the enabled channels: x (s12 in 16 bits, >>4) @0, y (u8) @2 -> 3 bytes
    xs, ys = [-5, 100, 7, -2048], [3, 250, 0, 9]
    data = b"".join(struct.pack("<HB", (x & 0xFFF) << 4, y) for x, y in zip(xs, ys))
    sysdir, devdir, dev = _fake_iio(str(tmp_path), data)
    p = nns.parse_launch(f"tensor_src_iio iio-base-dir={sysdir} dev-dir={devdir} device=fake_accel channels=0,1 "
                         "buffer-capacity=2 frequency=1000 ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).numpy("float32").copy()))
    p.run(timeout=20)
    caps = p.get_by_name("sink").pad_caps("sink")
    p.stop()
    assert len(out) == 2
    exp = np.array([[(x + 1) * 0.5, (y + 1) * 0.5] for x, y in zip(xs, ys)], np.float32)
    np.testing.assert_allclose(np.concatenate(out).reshape(4, 2), exp)
    assert caps.get("dimensions").startswith("2:2") and caps.get("framerate") == (1000, 2)
    # sysfs restored
    assert open(f"{dev}/scan_elements/in_accel_x_en").read() == "0"
    assert open(f"{dev}/buffer/enable").read() == "0"


def test_src_iio_unmerged_and_errors(nns, tmp_path):
    import struct
    # all channels: x @0, y @2, timestamp (s64) aligned @8 -> 16 bytes
    data = b"".join(struct.pack("<HB5xq", 16 * i, i, i) for i in range(3))
    sysdir, devdir, _ = _fake_iio(str(tmp_path), data)
    p = nns.parse_launch(f"tensor_src_iio iio-base-dir={sysdir} dev-dir={devdir} device-number=0 channels=all "
                         "merge-channels-data=false buffer-capacity=1 frequency=1000 ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.n_memory))
    p.run(timeout=20)
    p.stop()
    assert out == [3, 3, 3]
    p = nns.parse_launch(f"tensor_src_iio iio-base-dir={sysdir} dev-dir={devdir} device=nosuch ! fakesink")
    p.set_state("playing")
    msg = p.wait(10)
    p.stop()
    assert msg and msg[0] == "error"
