"""Element behaviour on the host path (reference: tests/nnstreamer_plugins/
unittest_plugins.cc, tests/transform_*/runTest.sh, nnstreamer_mux/merge/split/
demux/aggregator runTests)."""
import numpy as np
import pytest

from conftest import run_pipeline


def appsrc_pipeline(nns, tail, caps, frames, pts=None):
    p = nns.parse_launch(f"appsrc name=src caps={caps!r} ! {tail}".replace("'", '"'))
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b))
    p.set_state("playing")
    src = p.get_by_name("src")
    for i, f in enumerate(frames):
        src.push_buffer(f, pts=(pts[i] if pts else i * 1000000))
    src.end_of_stream()
    msg = p.wait(timeout=30)
    assert msg is not None and msg[0] == "eos", (msg, p.messages())
    p.stop()
    return out


# ------------------------------------------------------------ converter ----

def test_converter_video_rgb(nns):
    bufs = run_pipeline(nns, "videotestsrc num-buffers=2 pattern=gradient ! video/x-raw,format=RGB,width=16,height=8,"
                             "framerate=10/1 ! tensor_converter ! tensor_sink name=sink")
    assert len(bufs) == 2
    assert bufs[0].memory(0).size == 3 * 16 * 8
    assert bufs[1].pts == 100000000


def test_converter_strips_row_padding(nns):
    # width 5 RGB => stride 16 bytes (15 + pad 1): tensor must be 15 bytes per row
    p = nns.parse_launch("videotestsrc num-buffers=1 pattern=gradient ! video/x-raw,format=RGB,width=5,height=3 "
                         "! tee name=t t. ! queue ! appsink name=raw t. ! queue ! tensor_converter ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).numpy().copy()))
    raw = p.get_by_name("raw")
    p.set_state("playing")
    r = raw.pull(timeout=10).memory(0).numpy().copy()
    p.wait(10)
    p.stop()
    assert r.size == 16 * 3
    expect = np.concatenate([r[y * 16:y * 16 + 15] for y in range(3)])
    np.testing.assert_array_equal(out[0], expect)


def test_converter_frames_per_tensor(nns):
    frames = [np.full(12, i, np.uint8) for i in range(6)]
    out = appsrc_pipeline(nns, "tensor_converter input-dim=12 input-type=uint8 frames-per-tensor=3 ! tensor_sink name=sink",
                          "application/octet-stream", frames)
    assert len(out) == 2
    np.testing.assert_array_equal(out[1].memory(0).numpy(), np.repeat(np.arange(3, 6, dtype=np.uint8), 12))


def test_converter_octet_multi_tensor(nns):
    data = np.arange(8, dtype=np.uint8)
    out = appsrc_pipeline(nns, "tensor_converter input-dim=2:1,6 input-type=uint8,uint8 ! tensor_sink name=sink",
                          "application/octet-stream", [data])
    assert out[0].n_memory == 2
    np.testing.assert_array_equal(out[0].memory(1).numpy(), data[2:])


def test_converter_text(nns):
    out = appsrc_pipeline(nns, "tensor_converter input-dim=8 ! tensor_sink name=sink", "text/x-raw,format=utf8",
                          [b"hello", b"longer-than-8"])
    assert out[0].memory(0).bytes() == b"hello\0\0\0"
    assert out[1].memory(0).bytes() == b"longer-t"


def test_converter_audio(nns):
    pcm = np.arange(20, dtype=np.int16)
    out = appsrc_pipeline(nns, "tensor_converter frames-per-tensor=5 ! tensor_sink name=sink",
                          "audio/x-raw,format=S16LE,rate=8000,channels=2,layout=interleaved", [pcm])
    assert len(out) == 2
    np.testing.assert_array_equal(out[1].memory(0).numpy("int16"), pcm[10:])


def test_converter_flexible_to_static(nns):
    hdr = nns.meta_header(5, [4, 1], format=1)
    out = appsrc_pipeline(nns, "tensor_converter ! tensor_sink name=sink", "other/tensors,format=flexible,framerate=0/1",
                          [hdr + bytes([1, 2, 3, 4])])
    assert out[0].memory(0).bytes() == bytes([1, 2, 3, 4])


# ------------------------------------------------------------ transform ----

def _transform(nns, mode, option, arr, in_type, in_dim, extra=""):
    caps = f"other/tensors,format=static,num_tensors=1,dimensions={in_dim},types={in_type},framerate=0/1"
    out = appsrc_pipeline(nns, f"tensor_transform mode={mode} option={option} {extra} ! tensor_sink name=sink", caps, [arr])
    return out[0]


def test_transform_arithmetic_matches_numpy(nns):
    x = np.random.randint(0, 256, size=3 * 4 * 5, dtype=np.uint8)
    b = _transform(nns, "arithmetic", "typecast:float32,add:-127.5,div:127.5", x, "uint8", "3:4:5:1")
    np.testing.assert_allclose(b.memory(0).numpy("float32"), (x.astype(np.float32) - 127.5) / 127.5, rtol=1e-6)


def test_transform_arithmetic_int_wraps(nns):
    x = np.array([100, 120, -128, 5], dtype=np.int8)
    b = _transform(nns, "arithmetic", "add:100,mul:2", x, "int8", "4")
    ref = ((x.astype(np.int64) + 100).astype(np.int8).astype(np.int64) * 2).astype(np.int8)
    np.testing.assert_array_equal(b.memory(0).numpy("int8"), ref)


def test_transform_arithmetic_per_channel(nns):
    x = np.arange(12, dtype=np.float32)
    b = _transform(nns, "arithmetic", "per-channel:true@0,add:1@0,add:10@2,mul:2", x, "float32", "3:4")
    ref = x.reshape(4, 3).copy()
    ref[:, 0] += 1
    ref[:, 2] += 10
    ref *= 2
    np.testing.assert_allclose(b.memory(0).numpy("float32"), ref.ravel())


def test_transform_typecast(nns):
    x = np.array([1.7, -2.2, 300.0, 5.0], dtype=np.float32)
    b = _transform(nns, "typecast", "int16", x, "float32", "4")
    np.testing.assert_array_equal(b.memory(0).numpy("int16"), x.astype(np.int16))


def test_transform_transpose(nns):
    x = np.arange(3 * 4 * 5 * 2, dtype=np.float32)
    b = _transform(nns, "transpose", "1:2:0:3", x, "float32", "3:4:5:2")
    ref = x.reshape(2, 5, 4, 3).transpose(0, 3, 1, 2)  # NHWC -> NCHW
    np.testing.assert_array_equal(b.memory(0).numpy("float32"), ref.ravel())


def test_transform_dimchg(nns):
    x = np.arange(3 * 4 * 5, dtype=np.uint8)
    b = _transform(nns, "dimchg", "0:2", x, "uint8", "3:4:5:1")
    ref = x.reshape(5, 4, 3).transpose(2, 0, 1)
    np.testing.assert_array_equal(b.memory(0).numpy(), ref.ravel())


def test_transform_stand(nns):
    x = (np.random.rand(60) * 100).astype(np.float32)
    b = _transform(nns, "stand", "default", x, "float32", "3:20")
    ref = np.abs((x.astype(np.float64) - x.mean()) / x.std())
    np.testing.assert_allclose(b.memory(0).numpy("float32"), ref, rtol=1e-5, atol=1e-6)
    b = _transform(nns, "stand", "dc-average:float64,per-channel:true", x, "float32", "3:20")
    x64 = x.reshape(20, 3).astype(np.float64)
    r2 = (x64 - x64.mean(0)).ravel()
    np.testing.assert_allclose(b.memory(0).numpy("float64"), r2, rtol=1e-6)


def test_transform_clamp(nns):
    x = np.linspace(-5, 5, 11).astype(np.float32)
    b = _transform(nns, "clamp", "-1.5:2", x, "float32", "11")
    np.testing.assert_allclose(b.memory(0).numpy("float32"), np.clip(x, -1.5, 2))


def test_transform_apply_subset(nns):
    caps = "other/tensors,format=static,num_tensors=2,dimensions=2.2,types=uint8.uint8,framerate=0/1"
    out = appsrc_pipeline(nns, "tensor_transform mode=typecast option=float32 apply=1 ! tensor_sink name=sink", caps,
                          [[np.array([1, 2], np.uint8), np.array([3, 4], np.uint8)]])
    assert out[0].memory(0).size == 2 and out[0].memory(1).size == 8


def test_transform_bad_option(nns):
    with pytest.raises(Exception):
        nns.parse_launch("tensor_transform mode=transpose option=1:1:0:3")


# ---------------------------------------------------------- mux / demux ----

def test_mux_demux_roundtrip(nns):
    desc = ("videotestsrc num-buffers=3 pattern=red ! video/x-raw,format=RGB,width=4,height=4,framerate=30/1 "
            "! tensor_converter ! mux.sink_0 "
            "videotestsrc num-buffers=3 pattern=blue ! video/x-raw,format=GRAY8,width=4,height=4,framerate=30/1 "
            "! tensor_converter ! mux.sink_1 "
            "tensor_mux name=mux ! tensor_demux name=d tensorpick=1,0 d.src_0 ! queue ! tensor_sink name=sink "
            "d.src_1 ! queue ! fakesink")
    bufs = run_pipeline(nns, desc)
    assert len(bufs) == 3
    assert bufs[0].memory(0).size == 16  # GRAY8 picked first


def test_mux_caps_and_pts_slowest(nns):
    desc = ("videotestsrc num-buffers=4 ! video/x-raw,format=GRAY8,width=2,height=2,framerate=10/1 ! tensor_converter "
            "! mux.sink_0 videotestsrc num-buffers=8 ! video/x-raw,format=GRAY8,width=2,height=2,framerate=20/1 "
            "! tensor_converter ! mux.sink_1 tensor_mux name=mux sync-mode=slowest ! tensor_sink name=sink")
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.pts))
    p.run(timeout=30)
    caps = p.get_by_name("sink").pad_caps("sink")
    p.stop()
    assert caps.get("num_tensors") == 2
    assert out == sorted(out) and len(out) >= 3
    assert out[1] == 100000000


def test_merge_axis(nns):
    a = np.arange(6, dtype=np.float32)
    for axis, ref in [(0, np.concatenate([a.reshape(2, 3), a.reshape(2, 3) + 100], axis=1)),
                      (1, np.concatenate([a.reshape(2, 3), a.reshape(2, 3) + 100], axis=0))]:
        p = nns.parse_launch(
            f"appsrc name=a caps=other/tensors,format=static,num_tensors=1,dimensions=3:2,types=float32,framerate=0/1 ! m.sink_0 "
            f"appsrc name=b caps=other/tensors,format=static,num_tensors=1,dimensions=3:2,types=float32,framerate=0/1 ! m.sink_1 "
            f"tensor_merge name=m mode=linear option={axis} ! tensor_sink name=sink")
        out = []
        p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).numpy("float32").copy()))
        p.set_state("playing")
        p.get_by_name("a").push_buffer(a, pts=0)
        p.get_by_name("b").push_buffer(a + 100, pts=0)
        p.get_by_name("a").end_of_stream()
        p.get_by_name("b").end_of_stream()
        p.wait(10)
        p.stop()
        np.testing.assert_array_equal(out[0], ref.ravel())


def test_split(nns):
    x = np.arange(10, dtype=np.uint8)
    p = nns.parse_launch(
        "appsrc name=src caps=other/tensors,format=static,num_tensors=1,dimensions=10,types=uint8,framerate=0/1 "
        "! tensor_split name=s tensorseg=4,6 s.src_0 ! queue ! tensor_sink name=a s.src_1 ! queue ! tensor_sink name=b")
    oa, ob = [], []
    p.get_by_name("a").connect("new-data", lambda b: oa.append(b.memory(0).numpy().copy()))
    p.get_by_name("b").connect("new-data", lambda b: ob.append(b.memory(0).numpy().copy()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(x, pts=0)
    p.get_by_name("src").end_of_stream()
    p.wait(10)
    p.stop()
    np.testing.assert_array_equal(oa[0], x[:4])
    np.testing.assert_array_equal(ob[0], x[4:])


def test_aggregator_window_and_concat(nns):
    frames = [np.full(6, i, np.uint8) for i in range(5)]
    caps = "other/tensors,format=static,num_tensors=1,dimensions=3:2:1:1,types=uint8,framerate=10/1"
    out = appsrc_pipeline(nns, "tensor_aggregator frames-in=1 frames-out=2 frames-flush=1 frames-dim=1 "
                               "! tensor_sink name=sink", caps, frames)
    assert len(out) == 4
    got = out[0].memory(0).numpy().reshape(4, 3)
    np.testing.assert_array_equal(got[:2], 0)
    np.testing.assert_array_equal(got[2:], 1)


def test_aggregator_concat_middle_dim(nns):
    # frames 3:2:1:1 concatenated on dim 0 -> interleaved rows
    f0 = np.arange(6, dtype=np.uint8)
    f1 = np.arange(6, dtype=np.uint8) + 10
    caps = "other/tensors,format=static,num_tensors=1,dimensions=3:2,types=uint8,framerate=0/1"
    out = appsrc_pipeline(nns, "tensor_aggregator frames-out=2 frames-dim=0 ! tensor_sink name=sink", caps, [f0, f1])
    got = out[0].memory(0).numpy()
    ref = np.concatenate([f0.reshape(2, 3), f1.reshape(2, 3)], axis=1).ravel()
    np.testing.assert_array_equal(got, ref)


# ------------------------------------------------------------ misc / api ----

def test_launch_syntax_refs_and_caps(nns):
    desc = ("videotestsrc num-buffers=2 ! video/x-raw, format=(string)RGB, width=8, height=8 ! tee name=t "
            "t. ! queue ! tensor_converter ! tensor_sink name=sink t. ! queue ! fakesink")
    assert len(run_pipeline(nns, desc)) == 2


def test_launch_errors(nns):
    with pytest.raises(Exception):
        nns.parse_launch("no_such_element ! fakesink")
    with pytest.raises(Exception):
        nns.parse_launch("videotestsrc ! ! fakesink")
    with pytest.raises(Exception):
        nns.parse_launch("videotestsrc nosuchprop=1 ! fakesink")


def test_custom_easy_filter(nns):
    def double(inputs):
        return [inputs[0] * 2]

    nns.register_custom_easy("double_f32", double, [nns.TensorShape([4], np.float32)], [nns.TensorShape([4], np.float32)])
    caps = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"
    out = appsrc_pipeline(nns, "tensor_filter framework=custom-easy model=double_f32 ! tensor_sink name=sink", caps,
                          [np.array([1, 2, 3, 4], np.float32)])
    np.testing.assert_array_equal(out[0].memory(0).numpy("float32"), [2, 4, 6, 8])
    nns.unregister_custom_easy("double_f32")


def test_python3_filter_script(nns, workdir):
    path = f"{workdir}/scaler.py"
    with open(path, "w") as f:
        f.write(
            "import numpy as np\nimport nnstreamer_python as nns\n"
            "class CustomFilter(object):\n"
            "    def __init__(self, *args):\n        self.k = float(args[0]) if args else 1.0\n"
            "    def setInputDim(self, dims):\n        return [nns.TensorShape(dims[0].getDims(), np.float32)]\n"
            "    def invoke(self, arr):\n        return [arr[0].astype(np.float32) * self.k]\n")
    caps = "other/tensors,format=static,num_tensors=1,dimensions=3,types=uint8,framerate=0/1"
    out = appsrc_pipeline(nns, f"tensor_filter framework=python3 model={path} custom=3 ! tensor_sink name=sink", caps,
                          [np.array([1, 2, 3], np.uint8)])
    np.testing.assert_array_equal(out[0].memory(0).numpy("float32"), [3, 6, 9])


def test_filter_output_combination(nns):
    def inc(inputs):
        return [inputs[0] + 1]

    nns.register_custom_easy("inc_u8", inc, [nns.TensorShape([2], np.uint8)], [nns.TensorShape([2], np.uint8)])
    caps = "other/tensors,format=static,num_tensors=1,dimensions=2,types=uint8,framerate=0/1"
    out = appsrc_pipeline(nns, "tensor_filter framework=custom-easy model=inc_u8 output-combination=i0,o0 "
                               "! tensor_sink name=sink", caps, [np.array([5, 6], np.uint8)])
    assert out[0].n_memory == 2
    np.testing.assert_array_equal(out[0].memory(1).numpy(), [6, 7])


def test_image_labeling_cpu(nns, labels):
    caps = "other/tensors,format=static,num_tensors=1,dimensions=1000:1,types=float32,framerate=0/1"
    x = np.zeros(1000, np.float32)
    x[417] = 3.0
    x[900] = 3.0  # first max wins
    out = appsrc_pipeline(nns, f"tensor_decoder mode=image_labeling option1={labels} ! tensor_sink name=sink", caps, [x])
    assert out[0].memory(0).bytes() == b"class_417"


def test_direct_video_padding(nns):
    caps = "other/tensors,format=static,num_tensors=1,dimensions=3:5:2:1,types=uint8,framerate=0/1"
    x = np.arange(30, dtype=np.uint8)
    out = appsrc_pipeline(nns, "tensor_decoder mode=direct_video ! tensor_sink name=sink", caps, [x])
    got = out[0].memory(0).numpy()
    assert got.size == 16 * 2
    np.testing.assert_array_equal(got[:15], x[:15])
    np.testing.assert_array_equal(got[16:31], x[15:])
