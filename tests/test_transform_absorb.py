"""tensor_filter absorbs an adjacent upstream tensor_transform (runtime/fusion.h).

The reference classification string normalises in its own element
(`tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5`,
gsttensor_transform.c:1241-1412).  A model whose uint8 input goes through a
256-entry table (`in_lut`, the fused stems) takes that arithmetic into the table
at caps negotiation; the transform passes the uint8 frames through.  Outputs must
equal the unabsorbed pipeline's (transform kernel -> float32 model input), and
arithmetic the table cannot express keeps its own element.
"""
import os

import numpy as np
import pytest


@pytest.fixture(scope="module")
def fused_f32(workdir):
    from nnstreamer_amd.models.export import export

    return export("mobilenet_v2_fused_fp32", os.path.join(workdir, "mbv2_f32_absorb.pt"), layout="nhwc")


def _run(nns, model, transform, absorb=True, frames=2, dev=""):
    desc = (f"videotestsrc num-buffers={frames} pattern=snow ! video/x-raw,format=RGB,width=224,height=224,"
            f"framerate=30/1 ! tensor_converter frames-per-tensor={frames} {dev} "
            f"! {transform} ! tensor_filter name=f framework=pytorch model={model} input=3:224:224:{frames} "
            f"inputtype=float32 absorb-transform={'true' if absorb else 'false'} {dev} ! tensor_sink name=sink")
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).numpy("float32").copy()))
    p.run(timeout=300)
    info = (p.get_by_name("f").get_property("absorbed"), p.get_by_name("tt").get_property("absorbed-by"))
    p.stop()
    assert len(out) == 1
    return out[0], info


NORM = "tensor_transform name=tt mode=arithmetic option=typecast:float32,add:-127.5,div:127.5"


def test_reference_string_absorbed_bit_exact(nns, fused_f32):
    a, info = _run(nns, fused_f32, NORM, absorb=True)
    assert info == ("tt", "f")
    b, info_b = _run(nns, fused_f32, NORM, absorb=False)
    assert info_b == ("", "")
    # host path: the table holds the transform's own fp32 results -> identical model input
    np.testing.assert_array_equal(a, b)


def test_other_arithmetic_follows_the_transform(nns, fused_f32):
    tr = "tensor_transform name=tt mode=arithmetic option=typecast:float32,add:-100,mul:0.01"
    a, info = _run(nns, fused_f32, tr, absorb=True)
    assert info == ("tt", "f")
    b, _ = _run(nns, fused_f32, tr, absorb=False)
    np.testing.assert_array_equal(a, b)
    c, _ = _run(nns, fused_f32, NORM, absorb=True)
    assert not np.array_equal(a, c)  # the model's default table was replaced, not kept


@pytest.mark.parametrize("transform", [
    "tensor_transform name=tt mode=stand option=default:float32",
    "tensor_transform name=tt mode=arithmetic option=typecast:float32,per-channel:true@0,add:-127.5@0,div:127.5",
])
def test_non_absorbable_transform_keeps_its_kernel(nns, fused_f32, transform):
    _, info = _run(nns, fused_f32, transform, absorb=True)
    assert info == ("", "")


def test_plain_model_is_not_absorbed(nns, workdir):
    from nnstreamer_amd.models.export import export

    plain = export("mobilenet_v2", os.path.join(workdir, "mbv2_plain_absorb.pt"), layout="nhwc")
    _, info = _run(nns, plain, NORM, absorb=True)
    assert info == ("", "")


def test_lut_matches_transform_arithmetic():
    import torch

    from nnstreamer_amd.models.fused import input_lut

    v = torch.arange(256, dtype=torch.float32)
    ref = (v + np.float32(-127.5)) / np.float32(127.5)
    assert torch.equal(input_lut(-127.5, 127.5), ref)


def _run_labels(nns, model, workdir, absorb, frames=3, queue=True, dev=""):
    from nnstreamer_amd.models.export import write_labels

    labels = write_labels(os.path.join(workdir, "labels_absorb.txt"))
    q = "queue max-size-buffers=2 ! " if queue else ""
    desc = (f"videotestsrc num-buffers={frames} pattern=snow ! video/x-raw,format=RGB,width=224,height=224,"
            f"framerate=30/1 ! tensor_converter frames-per-tensor={frames} {dev} ! {NORM} "
            f"! tensor_filter name=f framework=pytorch model={model} input=3:224:224:{frames} inputtype=float32 "
            f"absorb-decoder={'true' if absorb else 'false'} {dev} ! {q}"
            f"tensor_decoder name=dec mode=image_labeling option1={labels} ! tensor_sink name=sink")
    p = nns.parse_launch(desc)
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(bytes(b.memory(0).bytes())))
    p.run(timeout=300)
    info = (p.get_by_name("f").get_property("absorbed-decoder"), p.get_by_name("dec").get_property("argmax-by"))
    p.stop()
    assert len(out) == 1
    return out[0].decode().split("\n"), info


@pytest.mark.parametrize("queue", [True, False])
def test_downstream_argmax_absorbed(nns, fused_f32, workdir, queue):
    """tensor_filter ! [queue !] tensor_decoder mode=image_labeling: the filter
    runs the decoder's argmax after its forward (int32 indices leave the model,
    runtime/fusion.h ArgmaxConsumer); labels equal the unabsorbed pipeline's."""
    a, info = _run_labels(nns, fused_f32, workdir, absorb=True, queue=queue)
    assert info == ("dec", "f")
    b, info_b = _run_labels(nns, fused_f32, workdir, absorb=False, queue=queue)
    assert info_b == ("", "")
    assert a == b and len(a) == 3
