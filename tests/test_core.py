"""Data model parity: dimension strings, types, meta headers, caps
(reference: gst/nnstreamer/nnstreamer_plugin_api_util_impl.c,
nnstreamer_plugin_api_impl.c; tests/common/unittest_common.cc)."""
import struct

import pytest


def test_parse_dimension_rank_and_defaults(nns):
    assert nns.parse_dimension("3:224:224:1") == (4, [3, 224, 224, 1, 1, 1, 1, 1])
    assert nns.parse_dimension("10") == (1, [10, 1, 1, 1, 1, 1, 1, 1])
    assert nns.parse_dimension(" 1 : 2 : 3 ")[0] == 3
    assert nns.parse_dimension("1:2:3:4:5:6:7:8")[1] == [1, 2, 3, 4, 5, 6, 7, 8]
    assert nns.parse_dimension("")[0] == 0


def test_dimension_strings(nns):
    assert nns.dimension_string([3, 4]) == "3:4:1:1:1:1:1:1"
    assert nns.dimension_string([3, 4, 5], rank=3) == "3:4:5"
    assert nns.dimension_string_equal("3:4:1:1", "3:4")
    assert nns.dimension_string_equal("3:4,5", "3:4:1,5:1")
    assert not nns.dimension_string_equal("3:4", "4:3")
    assert not nns.dimension_string_equal("3:4,5", "3:4")


@pytest.mark.parametrize("name,code,size", [
    ("int32", 0, 4), ("uint32", 1, 4), ("int16", 2, 2), ("uint16", 3, 2), ("int8", 4, 1), ("uint8", 5, 1),
    ("float64", 6, 8), ("float32", 7, 4), ("int64", 8, 8), ("uint64", 9, 8), ("float16", 10, 2), ("bfloat16", 12, 2),
])
def test_types(nns, name, code, size):
    assert nns.dtype_from_string(name) == code
    assert nns.dtype_from_string(name.upper()) == code
    assert nns.dtype_name(code) == name
    assert nns.dtype_size(code) == size


def test_unknown_type(nns):
    assert nns.dtype_from_string("int12") == 11
    assert nns.dtype_from_string("") == 11


def test_meta_header_layout(nns):
    h = nns.meta_header(7, [3, 224, 224, 1], format=1, media=0)
    assert len(h) == 128
    v = struct.unpack("<32I", h)
    assert v[0] == 0xDE001000 and v[1] == 7
    assert v[2:6] == (3, 224, 224, 1) and v[6] == 0
    assert v[18] == 1 and v[19] == 0 and v[20] == 0
    assert all(x == 0 for x in v[21:])
    d = nns.parse_meta_header(h)
    assert d["valid"] and d["header_size"] == 128 and d["data_size"] == 3 * 224 * 224 * 4


def test_meta_header_sparse_size(nns):
    h = nns.meta_header(5, [10, 10], format=2, nnz=7)
    d = nns.parse_meta_header(h)
    assert d["valid"] and d["nnz"] == 7 and d["data_size"] == 7 * (1 + 4)


def test_meta_header_invalid(nns):
    assert not nns.parse_meta_header(b"\0" * 128)["valid"]
    bad = bytearray(nns.meta_header(7, [1]))
    bad[8:12] = b"\0\0\0\0"  # dim[0] == 0
    assert not nns.parse_meta_header(bytes(bad))["valid"]


def test_caps_parse_and_print(nns):
    c = nns.Caps("other/tensors,format=static,num_tensors=1,dimensions=3:224:224:1,types=uint8,framerate=30/1")
    assert c.is_fixed()
    assert c.get("num_tensors") == 1
    assert c.get("framerate") == (30, 1)
    s = str(c)
    assert "dimensions=(string)3:224:224:1" in s and "framerate=(fraction)30/1" in s
    c2 = nns.Caps(s)
    assert str(c2) == s


def test_caps_intersect_dimension_spelling(nns):
    a = nns.Caps("other/tensors,format=static,num_tensors=1,dimensions=3:224:224:1,types=uint8,framerate=30/1")
    b = nns.Caps("other/tensors,format=static,num_tensors=1,dimensions=3:224:224,types=uint8")
    assert a.can_intersect(b)
    c = nns.Caps("other/tensors,format=static,num_tensors=1,dimensions=3:224:223,types=uint8")
    assert not a.can_intersect(c)


def test_caps_ranges_lists(nns):
    t = nns.Caps("video/x-raw,format={RGB,BGR},width=[1,4096],height=[1,4096],framerate=[0/1,2147483647/1]")
    f = nns.Caps("video/x-raw,format=BGR,width=640,height=480,framerate=30/1")
    i = t.intersect(f)
    assert i.is_fixed() and i.get("format") == "BGR" and i.get("width") == 640
    assert not t.can_intersect(nns.Caps("video/x-raw,format=GRAY8"))
    fx = t.fixate()
    assert fx.get("format") == "RGB" and fx.get("width") == 1


def test_caps_tensors_config(nns):
    c = nns.Caps("other/tensors,format=static,num_tensors=2,dimensions=3:4.5:6,types=float32.uint8,framerate=0/1")
    cfg = c.tensors_config()
    assert cfg["num_tensors"] == 2
    assert cfg["types"] == "float32,uint8"
    assert cfg["dimensions"].split(",")[1].startswith("5:6")
    legacy = nns.Caps("other/tensor,dimension=1:2:3,type=int16,framerate=5/1").tensors_config()
    assert legacy["num_tensors"] == 1 and legacy["types"] == "int16" and legacy["rate"] == (5, 1)


def test_caps_syntax_error(nns):
    with pytest.raises(Exception):
        nns.Caps("video/x-raw,width=(int")


def test_version_and_registry(nns):
    assert nns.version().startswith("nnsx")
    names = {e[0] for e in nns.list_elements()}
    for e in ["tensor_converter", "tensor_transform", "tensor_filter", "tensor_decoder", "tensor_sink",
              "tensor_mux", "tensor_demux", "tensor_merge", "tensor_split", "tensor_aggregator",
              "queue", "tee", "capsfilter", "videotestsrc", "appsrc", "appsink", "filesrc", "filesink"]:
        assert e in names, e
    assert "pytorch" in nns.subplugins("filter")
    assert "image_labeling" in nns.subplugins("decoder")


def test_extra_tensors_reference_layout(nns):
    """>16 tensors in the reference's buffer form: the 16th memory holds a
    GstTensorExtraInfo (nnstreamer_plugin_api_impl.c:1477-1490; LP64 layout:
    24-byte header + 200 x 48-byte GstTensorInfo) followed by tensor 15's and
    then every extra tensor's bytes.  appsrc accepts such buffers and hands one
    memory per tensor downstream."""
    import struct

    import numpy as np

    from nnstreamer_amd import _C

    n = 20
    arrays = [np.full(i + 1, i, np.uint8) for i in range(n)]
    dims = [f"{i + 1}" for i in range(n)]
    packed = _C.pack_extra(arrays, dims, ["uint8"] * n)
    assert len(packed) == 16
    blk = packed[15].numpy("uint8").tobytes()
    magic, version, num_extra, reserved = struct.unpack_from("<III4xQ", blk, 0)
    assert (magic, version, num_extra, reserved) == (0xF00DC0DE, 0, 4, 16)
    for k in range(200):
        name, typ = struct.unpack_from("<QI", blk, 24 + 48 * k)
        d = struct.unpack_from("<8I", blk, 24 + 48 * k + 12)
        assert name == 0
        if k < num_extra:
            assert typ == 5 and d[0] == 17 + k  # _NNS_UINT8, tensor 16 + k
        else:
            assert typ == 11  # _NNS_END (gst_tensor_info_init)
    off = 24 + 48 * 200
    assert off == 9624
    payload = blk[off:]
    assert payload == b"".join(a.tobytes() for a in arrays[15:])
    out, infos = _C.unpack_extra(list(packed))
    assert len(out) == n and [i for i, _ in infos] == [f"{k}:1:1:1:1:1:1:1" for k in range(17, 21)]
    for a, m in zip(arrays, out):
        np.testing.assert_array_equal(m.numpy("uint8"), a)

    caps = ('other/tensors,format=static,num_tensors=20,dimensions="' + ",".join(dims) + '",types="'
            + ",".join(["uint8"] * n) + '",framerate=0/1')
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_sink name=s")
    got = []
    p.get_by_name("s").connect("new-data", lambda b: got.append([b.memory(i).numpy("uint8").copy()
                                                                for i in range(b.n_memory)]))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(list(packed), pts=0)
    p.get_by_name("src").end_of_stream()
    assert p.wait(20)[0] == "eos", p.messages()
    p.stop()
    assert len(got) == 1 and len(got[0]) == n
    for a, m in zip(arrays, got[0]):
        np.testing.assert_array_equal(m, a)
