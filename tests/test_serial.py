"""protobuf / flatbuf / flexbuf decoders and converters (reference
tests/nnstreamer_{protobuf,flatbuf,flexbuf}/runTest.sh: tensors -> wire format
-> tensors must reproduce the raw frames).  Protobuf parity is pinned against
the Python protobuf runtime with the reference schema (nnstreamer.proto)
built at test time; flatbuf against a reader / writer written from the
FlatBuffers format rules for nnstreamer.fbs (tests/fbspec.py: no flatbuffers
library in this image, so not flatc's exact layout); flexbuf likewise
against tests/fxspec.py, whose writer uses the builder's narrowest slot
widths."""
import numpy as np
import pytest

WIRES = [("protobuf", "other/protobuf-tensor"), ("flatbuf", "other/flatbuf-tensor"), ("flexbuf", "other/flexbuf")]


def _collect(nns, desc, n=1):
    p = nns.parse_launch(desc)
    outs = []
    p.get_by_name("sink").connect("new-data", lambda b: outs.append([b.memory(i).bytes() for i in range(b.n_memory)]))
    p.run(timeout=30)
    return outs


@pytest.mark.parametrize("mode,caps", WIRES)
@pytest.mark.parametrize("fmt,w,h", [("RGB", 320, 240), ("BGRx", 64, 48), ("GRAY8", 33, 17)])
def test_roundtrip_video(nns, mode, caps, fmt, w, h):
    src = f"videotestsrc num-buffers=3 pattern=13 ! video/x-raw,format={fmt},width={w},height={h},framerate=5/1 ! tensor_converter"
    direct = _collect(nns, f"{src} ! tensor_sink name=sink")
    via = _collect(nns, f"{src} ! tensor_decoder mode={mode} ! {caps} ! tensor_converter ! tensor_sink name=sink")
    assert len(direct) == len(via) == 3
    assert direct == via


@pytest.mark.parametrize("mode,caps", WIRES)
def test_roundtrip_multi_tensor_and_caps(nns, mode, caps):
    desc = (f"tensor_mux name=mux ! tensor_decoder mode={mode} ! {caps} ! tensor_converter ! tensor_sink name=sink "
            "videotestsrc num-buffers=2 pattern=snow ! video/x-raw,format=RGB,width=8,height=4,framerate=5/1 "
            "! tensor_converter ! mux.sink_0 "
            "audiotestsrc num-buffers=2 samplesperbuffer=100 ! audio/x-raw,format=S16LE,channels=1,rate=500 "
            "! tensor_converter frames-per-tensor=100 ! mux.sink_1")
    p = nns.parse_launch(desc)
    got = []
    p.get_by_name("sink").connect("new-data", lambda b: got.append(b))
    p.run(timeout=30)
    assert len(got) == 2
    caps_str = str(p.get_by_name("sink").pad_caps("sink"))
    assert "num_tensors=(int)2" in caps_str and "uint8,int16" in caps_str and "3:8:4:1" in caps_str, caps_str
    assert got[0].memory(0).size == 96 and got[0].memory(1).size == 200


def _pb_classes():
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    fd = descriptor_pb2.FileDescriptorProto(name="nnstreamer_test.proto", package="nnstreamer.protobuf", syntax="proto3")
    t = fd.message_type.add(name="Tensor")
    t.field.add(name="name", number=1, type=9, label=1)
    en = t.enum_type.add(name="Tensor_type")
    for i, n in enumerate(["NNS_INT32", "NNS_UINT32", "NNS_INT16", "NNS_UINT16", "NNS_INT8", "NNS_UINT8",
                           "NNS_FLOAT64", "NNS_FLOAT32", "NNS_INT64", "NNS_UINT64"]):
        en.value.add(name=n, number=i)
    t.field.add(name="type", number=2, type=14, label=1, type_name=".nnstreamer.protobuf.Tensor.Tensor_type")
    t.field.add(name="dimension", number=3, type=13, label=3)
    t.field.add(name="data", number=4, type=12, label=1)
    ts = fd.message_type.add(name="Tensors")
    ts.field.add(name="num_tensor", number=1, type=13, label=1)
    fr = ts.nested_type.add(name="frame_rate")
    fr.field.add(name="rate_n", number=1, type=5, label=1)
    fr.field.add(name="rate_d", number=2, type=5, label=1)
    ts.field.add(name="fr", number=2, type=11, label=1, type_name=".nnstreamer.protobuf.Tensors.frame_rate")
    ts.field.add(name="tensor", number=3, type=11, label=3, type_name=".nnstreamer.protobuf.Tensor")
    ef = ts.enum_type.add(name="Tensor_format")
    for i, n in enumerate(["NNS_TENSOR_FORAMT_STATIC", "NNS_TENSOR_FORMAT_FLEXIBLE", "NNS_TENSOR_FORMAT_SPARSE"]):
        ef.value.add(name=n, number=i)
    ts.field.add(name="format", number=4, type=14, label=1, type_name=".nnstreamer.protobuf.Tensors.Tensor_format")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("nnstreamer.protobuf.Tensors"))


def test_protobuf_bytes_match_protobuf_runtime(nns):
    Tensors = _pb_classes()
    out = _collect(nns, "videotestsrc num-buffers=1 pattern=snow ! video/x-raw,format=RGB,width=6,height=5,framerate=5/1 "
                        "! tensor_converter ! tensor_decoder mode=protobuf ! tensor_sink name=sink")
    blob = out[0][0]
    msg = Tensors()
    msg.ParseFromString(blob)
    assert msg.num_tensor == 1 and msg.fr.rate_n == 5 and msg.fr.rate_d == 1
    t = msg.tensor[0]
    assert t.type == 5 and list(t.dimension)[:4] == [3, 6, 5, 1] and len(t.data) == 90
    # canonical serialization by the protobuf runtime is byte-identical
    assert msg.SerializeToString() == blob


def test_protobuf_runtime_message_converts(nns):
    Tensors = _pb_classes()
    msg = Tensors(num_tensor=2, format=0)
    msg.fr.rate_n, msg.fr.rate_d = 30, 1
    a = np.arange(12, dtype=np.float32)
    b = np.arange(6, dtype=np.int64) - 3
    msg.tensor.add(name="a", type=7, dimension=[4, 3, 1, 1, 0, 0, 0, 0], data=a.tobytes())
    msg.tensor.add(name="b", type=8, dimension=[6], data=b.tobytes())
    p = nns.parse_launch("appsrc name=src caps=other/protobuf-tensor,framerate=30/1 ! tensor_converter "
                         "! tensor_sink name=sink")
    got = []
    p.get_by_name("sink").connect("new-data", lambda buf: got.append(buf))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(msg.SerializeToString(), pts=0)
    p.get_by_name("src").end_of_stream()
    assert p.wait(20)[0] == "eos"
    caps = str(p.get_by_name("sink").pad_caps("sink"))
    p.stop()
    np.testing.assert_array_equal(got[0].memory(0).numpy("float32"), a)
    np.testing.assert_array_equal(got[0].memory(1).numpy("int64"), b)
    assert "float32,int64" in caps and "4:3" in caps and "framerate=(fraction)30/1" in caps, caps


@pytest.mark.parametrize("mode,caps", WIRES)
def test_malformed_input_errors(nns, mode, caps):
    p = nns.parse_launch(f"appsrc name=src caps={caps},framerate=0/1 ! tensor_converter ! tensor_sink name=sink")
    p.set_state("playing")
    p.get_by_name("src").push_buffer(b"\x07\x01garbage-not-a-valid-frame", pts=0)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(20)
    p.stop()
    assert msg and msg[0] == "error"


def test_flatbuf_bytes_read_by_spec_reader(nns):
    """tensor_decoder mode=flatbuf output read by a FlatBuffers reader written from
    the format rules (tests/fbspec.py), field by field against nnstreamer.fbs
    (tensordec-flatbuf.cc:57-121 writes num_tensor, fr, tensor[name, type,
    dimension, data], format)"""
    from fbspec import Reader

    src = "videotestsrc num-buffers=1 pattern=snow ! video/x-raw,format=RGB,width=6,height=5,framerate=5/1 ! tensor_converter"
    raw = _collect(nns, f"{src} ! tensor_sink name=sink")[0][0]
    blob = _collect(nns, f"{src} ! tensor_decoder mode=flatbuf ! tensor_sink name=sink")[0][0]
    m = Reader(blob).tensors()
    assert m["num_tensor"] == 1 and m["fr"] == (5, 1) and m["format"] == 0
    t = m["tensor"][0]
    assert t["type"] == 5  # NNS_UINT8
    # NNS_TENSOR_RANK_LIMIT entries; the ranks past the caps' dimension string are 1, as
    # gst_tensor_parse_dimension fills them (nnstreamer_plugin_api_util_impl.c:949-950)
    assert t["dims"] == [3, 6, 5, 1, 1, 1, 1, 1]
    assert t["data"] == bytes(raw)


@pytest.mark.parametrize("shared_vtable", [True, False])
def test_flatbuf_spec_writer_layouts_convert(nns, shared_vtable):
    """tensor_converter on flatbuffers laid out unlike our encoder: vtables after
    their tables (negative soffset) or shared by every Tensor table, inline fields
    out of schema order, children in another order, and an unknown trailing field
    (a newer schema's) -- every valid layout must decode to the same tensors"""
    from fbspec import Writer

    a = np.arange(12, dtype=np.float32) * 0.5
    b = np.arange(6, dtype=np.int64) - 3
    blob = Writer().build([dict(name="a", type=7, dims=[4, 3, 1, 1], data=a.tobytes()),
                           dict(name="bee", type=8, dims=[6, 1, 1, 1], data=b.tobytes())],
                          fr=(30, 1), shared_vtable=shared_vtable)
    p = nns.parse_launch("appsrc name=src caps=other/flatbuf-tensor,framerate=30/1 ! tensor_converter "
                         "! tensor_sink name=sink")
    got = []
    p.get_by_name("sink").connect("new-data", lambda buf: got.append(buf))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(blob, pts=0)
    p.get_by_name("src").end_of_stream()
    assert p.wait(20)[0] == "eos", p.messages()
    caps = str(p.get_by_name("sink").pad_caps("sink"))
    p.stop()
    np.testing.assert_array_equal(got[0].memory(0).numpy("float32"), a)
    np.testing.assert_array_equal(got[0].memory(1).numpy("int64"), b)
    assert "float32,int64" in caps and "4:3" in caps and "framerate=(fraction)30/1" in caps, caps


def test_flexbuf_bytes_read_by_spec_reader(nns):
    """tensor_decoder mode=flexbuf output read by a FlexBuffers reader written from
    the format rules (tests/fxspec.py): the map tensordec-flexbuf.cc:120-160 builds"""
    from fxspec import Reader

    src = "videotestsrc num-buffers=1 pattern=snow ! video/x-raw,format=RGB,width=6,height=5,framerate=5/1 ! tensor_converter"
    raw = _collect(nns, f"{src} ! tensor_sink name=sink")[0][0]
    blob = _collect(nns, f"{src} ! tensor_decoder mode=flexbuf ! tensor_sink name=sink")[0][0]
    m = Reader(blob).root()
    assert sorted(m) == ["format", "num_tensors", "rate_d", "rate_n", "tensor_0"]
    assert (m["num_tensors"], m["rate_n"], m["rate_d"], m["format"]) == (1, 5, 1, 0)
    name, typ, dims, data = m["tensor_0"]
    assert name == "" and typ == 5 and dims == [3, 6, 5, 1, 1, 1, 1, 1] and data == bytes(raw)


@pytest.mark.parametrize("n", [12, 40000])
def test_flexbuf_narrow_widths_convert(nns, n):
    """tensor_converter on FlexBuffers with the builder's narrowest slot widths
    (1-byte maps and vectors for small tensors, wider ones past 255 / 65535) --
    what the reference's decoder emits -- where our encoder writes 8-byte slots"""
    from fxspec import Writer

    a = np.arange(n, dtype=np.float32) * 0.25
    b = (np.arange(6, dtype=np.int64) - 3) * 1000
    blob = Writer().build([dict(name="a", type=7, dims=[n, 1, 1, 1, 1, 1, 1, 1], data=a.tobytes()),
                           dict(name="b", type=8, dims=[6, 1, 1, 1, 1, 1, 1, 1], data=b.tobytes())], rate=(30, 1))
    p = nns.parse_launch("appsrc name=src caps=other/flexbuf,framerate=30/1 ! tensor_converter ! tensor_sink name=sink")
    got = []
    p.get_by_name("sink").connect("new-data", lambda buf: got.append(buf))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(blob, pts=0)
    p.get_by_name("src").end_of_stream()
    assert p.wait(20)[0] == "eos", p.messages()
    caps = str(p.get_by_name("sink").pad_caps("sink"))
    p.stop()
    np.testing.assert_array_equal(got[0].memory(0).numpy("float32"), a)
    np.testing.assert_array_equal(got[0].memory(1).numpy("int64"), b)
    assert "float32,int64" in caps and "framerate=(fraction)30/1" in caps, caps
