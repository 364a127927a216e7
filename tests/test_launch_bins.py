"""gst-launch bins: `( ... )` and `<type>.( ... )` groups with their own name=,
linked like gst-launch links a bin's ghost pads (reference
tools/development/parser/grammar.y bin rules).  nnsx flattens them."""
import numpy as np
import pytest


def _collect(p, name="sink"):
    out = []
    p.get_by_name(name).connect("new-data", lambda b: out.append(b.memory(0).numpy("uint8").copy()))
    return out


def test_bin_linked_on_both_sides(nns):
    p = nns.parse_launch("videotestsrc num-buffers=3 pattern=red ! video/x-raw,format=RGB,width=4,height=2,"
                         "framerate=30/1 ! ( name=conv tensor_converter ! queue ) ! tensor_sink name=sink")
    out = _collect(p)
    p.run(timeout=20)
    p.stop()
    assert len(out) == 3 and out[0].size == 24 and out[0][0] == 255


def test_bin_typed_and_nested_with_named_reference(nns):
    p = nns.parse_launch("videotestsrc num-buffers=2 pattern=blue ! video/x-raw,format=RGB,width=4,height=2,"
                         "framerate=30/1 ! tee name=t "
                         "bin.( name=b1 queue ! ( tensor_converter ! tensor_transform mode=typecast option=uint8 ) ) "
                         "! tensor_sink name=sink t. ! b1.")
    out = _collect(p)
    p.run(timeout=20)
    p.stop()
    assert len(out) == 2 and out[0][2] == 255


def test_bin_without_spaces_and_chains_after(nns):
    p = nns.parse_launch("(videotestsrc num-buffers=1 pattern=white ! video/x-raw,format=RGB,width=2,height=2,"
                         "framerate=30/1 ! tensor_converter) ! tensor_sink name=sink")
    out = _collect(p)
    p.run(timeout=20)
    p.stop()
    assert len(out) == 1 and out[0].tolist() == [255] * 12


@pytest.mark.parametrize("desc", ["( videotestsrc ! fakesink", "videotestsrc ! fakesink )", "( ) ! fakesink"])
def test_bin_syntax_errors(nns, desc):
    with pytest.raises(Exception):
        nns.parse_launch(desc)
