"""Device paths of tensor_sparse_enc / tensor_sparse_dec (K21, kernels/sparse.hip)
and tensor_if TENSOR_AVERAGE_VALUE (K22) against their host oracles: the same
pipeline with the tensors kept in host memory.  Device residency comes from an
upstream `tensor_transform ... device=0` (identity arithmetic on the GPU: mul:1 keeps -0.0)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TYPES = {"uint8": np.uint8, "int16": np.int16, "float32": np.float32, "float64": np.float64, "int64": np.int64}


def _sparse_run(nns, arr, tname, device):
    dims = ":".join(str(d) for d in reversed(arr.shape))
    caps = f"other/tensors,format=static,num_tensors=1,dimensions={dims},types={tname},framerate=0/1"
    up = "! tensor_transform mode=arithmetic option=mul:1 device=0 " if device else ""
    p = nns.parse_launch(f"appsrc name=src caps={caps} {up}! tensor_sparse_enc ! tee name=t "
                         "t. ! queue ! tensor_sink name=enc t. ! queue ! tensor_sparse_dec ! tensor_sink name=dec")
    enc, dec = [], []
    p.get_by_name("enc").connect("new-data", lambda b: enc.append(b.memory(0).bytes()))
    p.get_by_name("dec").connect("new-data", lambda b: dec.append(b.memory(0).numpy(tname).copy()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(arr, pts=0)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(60)
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    return enc[0], dec[0]


@pytest.mark.parametrize("tname", list(TYPES))
@pytest.mark.parametrize("shape,density", [((7,), 0.5), ((64, 64), 0.1), ((3, 4099), 0.3), ((256, 1024), 0.01),
                                           ((33, 65, 3), 0.0), ((5000,), 1.0)])
def test_sparse_device_bytes_equal_host(nns, tname, shape, density):
    rng = np.random.default_rng(hash((tname, shape)) & 0xffff)
    dt = TYPES[tname]
    vals = (rng.integers(1, 100, size=shape) * (1 if np.issubdtype(dt, np.integer) else 0.37)).astype(dt)
    arr = np.where(rng.random(shape) < density, vals, 0).astype(dt)
    enc_h, dec_h = _sparse_run(nns, arr, tname, device=False)
    enc_d, dec_d = _sparse_run(nns, arr, tname, device=True)
    assert enc_d == enc_h  # header + values + indices, byte for byte
    np.testing.assert_array_equal(dec_d.reshape(-1), arr.reshape(-1))
    np.testing.assert_array_equal(dec_h.reshape(-1), arr.reshape(-1))


def test_sparse_negative_zero_is_nonzero_on_device(nns):
    arr = np.array([0.0, -0.0, 1.0, 0.0], np.float32)
    enc_h, _ = _sparse_run(nns, arr, "float32", device=False)
    enc_d, dec_d = _sparse_run(nns, arr, "float32", device=True)
    assert enc_d == enc_h and nns.parse_meta_header(enc_d[:128])["nnz"] == 2
    assert np.signbit(dec_d[1])


def _if_avg(nns, arr, tname, sv, device):
    dims = ":".join(str(d) for d in reversed(arr.shape))
    caps = f"other/tensors,format=static,num_tensors=1,dimensions={dims},types={tname},framerate=0/1"
    up = "! tensor_transform mode=arithmetic option=mul:1 device=0 " if device else ""
    p = nns.parse_launch(f"appsrc name=src caps={caps} {up}! tensor_if name=tif compared-value=TENSOR_AVERAGE_VALUE "
                         f"compared-value-option=0 supplied-value={sv} operator=GT then=PASSTHROUGH else=PASSTHROUGH "
                         "tif.src_0 ! queue ! tensor_sink name=t tif.src_1 ! queue ! tensor_sink name=f")
    got = {"t": 0, "f": 0}
    p.get_by_name("t").connect("new-data", lambda b: got.__setitem__("t", got["t"] + 1))
    p.get_by_name("f").connect("new-data", lambda b: got.__setitem__("f", got["f"] + 1))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(arr, pts=0)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(60)
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    return got["t"] == 1


@pytest.mark.parametrize("tname,n", [("float32", 1 << 20), ("uint8", 3 * 224 * 224), ("int16", 1000), ("float64", 77)])
def test_if_average_device_matches_host(nns, tname, n):
    rng = np.random.default_rng(n)
    dt = TYPES[tname]
    arr = (rng.random(n) * 200).astype(dt)
    mean = float(arr.astype(np.float64).mean())
    for sv in (mean - 1, mean + 1, round(mean) - 1, round(mean) + 1):
        assert _if_avg(nns, arr, tname, f"{sv:.6f}", True) == _if_avg(nns, arr, tname, f"{sv:.6f}", False), sv
