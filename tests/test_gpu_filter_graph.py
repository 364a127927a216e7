"""tensor_filter framework=pytorch under hipGraph on the GPU: hot reload while
earlier outputs are still queued downstream (the re-capture must not be
disturbed by the releases of those outputs, which make the element stream wait
for their readers; csrc/filter/pytorch.cc graph_for)."""
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Scale(torch.nn.Module):
    def __init__(self, k: float):
        super().__init__()
        self.k = k

    def forward(self, x):
        return x * self.k + 1.0


def test_hipgraph_hot_reload_with_queued_outputs(nns, tmp_path):
    a, b = tmp_path / "a.pt", tmp_path / "b.pt"
    torch.jit.script(_Scale(2.0)).save(str(a))
    torch.jit.script(_Scale(3.0)).save(str(b))
    n = 4096
    caps = f"other/tensors,format=static,num_tensors=1,dimensions={n},types=float32,framerate=0/1"
    p = nns.parse_launch(
        f"appsrc name=src caps={caps} ! tensor_filter name=f framework=pytorch model={a} is-updatable=true "
        "accelerator=true:gpu device=0 custom=hipgraph:true ! queue max-size-buffers=16 ! tensor_sink name=s")
    got = []
    gate = {"slow": True}

    def on_data(buf):
        if gate["slow"]:
            time.sleep(0.02)  # a slow consumer: outputs pile up in the queue
        got.append(float(buf.memory(0).numpy("float32")[0]))

    p.get_by_name("s").connect("new-data", on_data)
    p.set_state("playing")
    src = p.get_by_name("src")
    for i in range(8):
        src.push_buffer(np.full(n, 1.0, np.float32), pts=i)
    t0 = time.time()
    while len(got) < 8 and time.time() - t0 < 20:  # model A must be done with all 8 before the swap
        time.sleep(0.005)
    assert len(got) == 8, got
    # swap the model while fresh frames keep the graph path busy and outputs queue up
    for i in range(8, 12):
        src.push_buffer(np.full(n, 1.0, np.float32), pts=i)
    time.sleep(0.05)
    p.get_by_name("f").set_property("model", str(b))
    for i in range(12, 24):
        src.push_buffer(np.full(n, 1.0, np.float32), pts=i)
    gate["slow"] = False
    src.end_of_stream()
    assert p.wait(60)[0] == "eos", p.messages()
    p.stop()
    assert len(got) == 24, got
    assert got[:8] == [3.0] * 8
    # frames 8..11 raced the swap (A or B); every later frame saw model B
    assert all(v in (3.0, 4.0) for v in got[8:12]), got
    assert got[12:] == [4.0] * 12, got


@pytest.mark.parametrize("upload", ["appsrc", "converter"])
def test_hipgraph_static_outputs_never_overwritten_while_held(nns, tmp_path, upload):
    """Copy-free graph outputs: a static output is handed downstream only while
    no earlier one is still held; with a slow consumer behind a deep queue every
    frame must still carry its own result (graph instances whose outputs are
    held are not replayed).  upload=converter feeds the filter from
    tensor_converter's device buffers."""
    m = tmp_path / "m.pt"
    torch.jit.script(_Scale(2.0)).save(str(m))
    n = 3 * 16 * 8
    frames = [np.full(n, i % 251, np.uint8) for i in range(40)]
    caps = "other/tensors,format=static,num_tensors=1,dimensions=3:16:8:1,types=uint8,framerate=0/1"
    video = "video/x-raw,format=RGB,width=16,height=8,framerate=0/1"
    head = (f"appsrc name=src caps={video} ! tensor_converter device=0 " if upload == "converter"
            else f"appsrc name=src caps={caps} ")
    p = nns.parse_launch(
        head + f"! tensor_transform mode=typecast option=float32 ! tensor_filter framework=pytorch model={m} "
        "accelerator=true:gpu device=0 custom=hipgraph:true ! queue max-size-buffers=32 ! tensor_sink name=s")
    got = []

    def on_data(buf):
        if len(got) < 20:
            time.sleep(0.01)  # slow at first: outputs stay held in the queue
        got.append(buf.memory(0).numpy("float32").copy())

    p.get_by_name("s").connect("new-data", on_data)
    p.set_state("playing")
    src = p.get_by_name("src")
    for i, f in enumerate(frames):
        src.push_buffer(f, pts=i)
    src.end_of_stream()
    assert p.wait(60)[0] == "eos", p.messages()
    p.stop()
    assert len(got) == len(frames)
    for i, g in enumerate(got):
        np.testing.assert_array_equal(g, np.full(n, 2.0 * (i % 251) + 1.0, np.float32), err_msg=f"frame {i}")
