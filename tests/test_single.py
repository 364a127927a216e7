"""Single-shot API (ML API "single"; reference tests/capi/unittest_capi_inference_single.cc
patterns: open with/without info, invoke, wrong input size, set_input_info,
timeout, close)."""
import textwrap
import time

import numpy as np
import pytest
import torch


def _export_linear(path, din=4, dout=3, seed=0):
    torch.manual_seed(seed)
    m = torch.nn.Linear(din, dout).eval()
    torch.jit.script(m).save(str(path))
    return m


def test_custom_easy_single(nns):
    nns.register_custom_easy("single_double", lambda x: [x[0] * 2],
                             [nns.TensorShape([4], np.float32)], [nns.TensorShape([4], np.float32)])
    with nns.Single("single_double", framework="custom-easy") as s:
        assert [t.getDims()[0] for t in s.input_info] == [4]
        (y,) = s.invoke(np.arange(4, dtype=np.float32))
        np.testing.assert_array_equal(y, 2 * np.arange(4, dtype=np.float32))
        with pytest.raises(Exception):
            s.invoke(np.arange(5, dtype=np.float32))  # wrong size
    nns.unregister_custom_easy("single_double")


def test_pytorch_single_cpu_auto_framework(nns, tmp_path):
    m = _export_linear(tmp_path / "lin.pt")
    x = np.random.default_rng(0).standard_normal((2, 4)).astype(np.float32)
    with nns.Single(str(tmp_path / "lin.pt"), input=[nns.TensorShape([4, 2], np.float32)],
                    output=[nns.TensorShape([3, 2], np.float32)], accelerator="false") as s:
        assert s.framework == "pytorch" and s.device == -1
        (y,) = s.invoke(x)
        np.testing.assert_allclose(y, m(torch.from_numpy(x)).detach().numpy(), rtol=1e-5, atol=1e-6)


def test_pytorch_single_set_input_info(nns, tmp_path):
    m = _export_linear(tmp_path / "lin.pt")
    s = nns.Single(str(tmp_path / "lin.pt"), framework="pytorch", input=[nns.TensorShape([4, 1], np.float32)],
                   accelerator="false")
    x = np.ones((1, 4), np.float32)
    (y,) = s.invoke(x)
    assert y.size == 3
    s.set_input_info([nns.TensorShape([4, 5], np.float32)])
    assert s.input_info[0].getDims()[:2] == [4, 5]
    x5 = np.random.default_rng(1).standard_normal((5, 4)).astype(np.float32)
    ys, info = s.invoke_dynamic(x5)
    assert info[0].getDims()[:2] == [3, 5]
    np.testing.assert_allclose(ys[0].reshape(5, 3), m(torch.from_numpy(x5)).detach().numpy(), rtol=1e-5, atol=1e-6)
    s.close()
    with pytest.raises(Exception):
        s.invoke(x)  # closed


def test_single_timeout(nns):
    def slow(x):
        time.sleep(0.6)
        return [x[0]]

    nns.register_custom_easy("single_slow", slow, [nns.TensorShape([2], np.int32)], [nns.TensorShape([2], np.int32)])
    s = nns.Single("single_slow", framework="custom-easy", timeout_ms=100)
    with pytest.raises(TimeoutError):
        s.invoke(np.array([1, 2], np.int32))
    s.timeout = 5000
    (y,) = s.invoke(np.array([3, 4], np.int32))  # waits for the late one, then runs
    assert y.tolist() == [3, 4]
    s.close()
    nns.unregister_custom_easy("single_slow")


def test_python3_single(nns, tmp_path):
    script = tmp_path / "f.py"
    script.write_text(textwrap.dedent("""
        import numpy as np
        import nnstreamer_python as nns
        class CustomFilter:
            def __init__(self, *args):
                self.i = [nns.TensorShape([3], np.float32)]
            def getInputDim(self):
                return self.i
            def getOutputDim(self):
                return self.i
            def invoke(self, x):
                return [x[0] + 1]
    """))
    with nns.Single(str(script), framework="python3") as s:
        (y,) = s.invoke(np.zeros(3, np.float32))
        np.testing.assert_array_equal(y, np.ones(3, np.float32))


def test_missing_model_fails(nns, tmp_path):
    with pytest.raises(Exception):
        nns.Single(str(tmp_path / "nope.pt"), framework="pytorch")


@pytest.mark.gpu
def test_pytorch_single_gpu_zero_copy(nns, tmp_path):
    m = _export_linear(tmp_path / "lin.pt", 8, 6)
    s = nns.Single(str(tmp_path / "lin.pt"), input=[nns.TensorShape([8, 16], np.float32)], accelerator="true:gpu",
                   device=0)
    assert s.device == 0
    x = torch.randn(16, 8, device="cuda")
    (y,) = s.invoke(x, output="torch")
    assert y.is_cuda
    torch.testing.assert_close(y.reshape(16, 6), m.cuda()(x), rtol=1e-4, atol=1e-4)
    (yn,) = s.invoke(x.cpu().numpy())
    np.testing.assert_allclose(yn.reshape(16, 6), m.cuda()(x).detach().cpu().numpy(), rtol=1e-4, atol=1e-4)
    s.close()


class _Scale(torch.nn.Module):
    def __init__(self, k: float):
        super().__init__()
        self.k = k

    def forward(self, x):
        return x * self.k


def test_pytorch_hot_reload_mid_stream(nns, tmp_path):
    """is-updatable + a new model= while PLAYING (tensor_filter_common.c:1404-1462):
    frames before the swap see model A, frames after it model B, none is lost."""
    a, b = tmp_path / "a.pt", tmp_path / "b.pt"
    torch.jit.script(_Scale(2.0)).save(str(a))
    torch.jit.script(_Scale(3.0)).save(str(b))
    caps = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_filter name=f framework=pytorch model={a} "
                         "is-updatable=true accelerator=false ! tensor_sink name=s")
    got = []
    p.get_by_name("s").connect("new-data", lambda buf: got.append(float(buf.memory(0).numpy("float32")[0])))
    p.set_state("playing")
    src = p.get_by_name("src")
    for i in range(3):
        src.push_buffer(np.ones(4, np.float32), pts=i)
    import time
    t0 = time.time()
    while len(got) < 3 and time.time() - t0 < 10:
        time.sleep(0.01)
    p.get_by_name("f").set_property("model", str(b))
    for i in range(3, 6):
        src.push_buffer(np.ones(4, np.float32), pts=i)
    src.end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    p.stop()
    assert got == [2.0, 2.0, 2.0, 3.0, 3.0, 3.0]
