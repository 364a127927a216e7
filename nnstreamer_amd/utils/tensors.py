"""Tensor helpers shared by the Python API, the `nnstreamer_python` script
module (reference API: ``nns.TensorShape(dims, np_dtype)``) and the tests."""
from __future__ import annotations

import numpy as np

# NNStreamer type enum order (tensor_typedef.h:133-148) + nnsx bfloat16 (12)
DTYPES = ["int32", "uint32", "int16", "uint16", "int8", "uint8", "float64", "float32", "int64", "uint64", "float16"]
NP_TYPES = {
    "int32": np.int32,
    "uint32": np.uint32,
    "int16": np.int16,
    "uint16": np.uint16,
    "int8": np.int8,
    "uint8": np.uint8,
    "float64": np.float64,
    "float32": np.float32,
    "int64": np.int64,
    "uint64": np.uint64,
    "float16": np.float16,
}


class TensorShape:
    """One tensor's dims (innermost first, as NNStreamer) and numpy dtype."""

    def __init__(self, dims, dtype):
        self._dims = [int(d) for d in dims]
        self._type = np.dtype(dtype)

    def getDims(self):  # noqa: N802  (reference API)
        return list(self._dims)

    def getType(self):  # noqa: N802
        return self._type

    def __repr__(self):
        return f"TensorShape({self._dims}, {self._type})"


def parse_caps_config(caps):
    """Return (types, dims) lists from an other/tensors caps object or string."""
    from .. import _C

    if isinstance(caps, str):
        caps = _C.Caps(caps)
    cfg = caps.tensors_config()
    if cfg is None:
        return [], []
    types = [t for t in cfg["types"].split(",") if t]
    dims = []
    for d in cfg["dimensions"].split(","):
        if d:
            dims.append([int(x) for x in d.split(":")])
    return types, dims


def to_numpy(mem, dtype="uint8", dims=None):
    """Memory -> numpy array; `dims` innermost-first (NNStreamer order)."""
    arr = mem.numpy(dtype)
    if dims:
        shape = [int(d) for d in dims][::-1]
        arr = arr.reshape(shape)
    return arr


def to_torch(mem, dtype="float32", dims=None):
    """Memory -> torch tensor, zero-copy via DLPack (device memories stay on the GPU)."""
    import torch

    if dims is None:
        n = mem.size // np.dtype(NP_TYPES.get(dtype, np.uint8)).itemsize if dtype != "bfloat16" else mem.size // 2
        dims = [n]
    cap = mem.dlpack(dtype, [int(d) for d in dims])
    return torch.from_dlpack(cap)
