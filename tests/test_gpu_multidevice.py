"""One pipeline across two GPUs of one process (branch data parallelism inside
a pipeline): a tee fans the frames out to a tensor_filter on device=0 and one
on device=1, tensor_mux joins the branches.  The device-1 branch's input is
moved by the peer-to-peer path (Memory::map_device -> hipMemcpyPeerAsync over
xGMI) and the mux pulls device-1 outputs back beside device-0 ones.  Needs two
GPUs: skipped on one-GPU boxes."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


class _Affine(torch.nn.Module):
    def forward(self, x):
        return x * 2.0 + 1.0


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs")
def test_tee_two_devices_mux(nns, tmp_path):
    model = tmp_path / "affine.pt"
    torch.jit.script(_Affine()).save(str(model))
    caps = "other/tensors,format=static,num_tensors=1,dimensions=1024,types=float32,framerate=0/1"
    p = nns.parse_launch(
        f"appsrc name=src caps={caps} ! tensor_transform mode=arithmetic option=mul:1 device=0 ! tee name=t "
        f"t. ! queue ! tensor_filter framework=pytorch model={model} accelerator=true:gpu device=0 ! mux.sink_0 "
        f"t. ! queue ! tensor_filter framework=pytorch model={model} accelerator=true:gpu device=1 ! mux.sink_1 "
        "tensor_mux name=mux sync-mode=nosync ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(
        [(b.memory(i).device, b.memory(i).numpy("float32").copy()) for i in range(b.n_memory)]))
    p.set_state("playing")
    frames = [np.full(1024, i, np.float32) for i in range(5)]
    for i, f in enumerate(frames):
        p.get_by_name("src").push_buffer(f, pts=i)
    p.get_by_name("src").end_of_stream()
    assert p.wait(60)[0] == "eos", p.messages()
    p.stop()
    assert len(out) == 5
    for f, mems in zip(frames, out):
        assert len(mems) == 2 and all(d in (0, 1) for d, _ in mems)  # outputs stay in HBM
        for _, v in mems:
            np.testing.assert_array_equal(v, f * 2 + 1)
