"""Single-shot inference: the ML API "single" (``ml_single_open`` /
``ml_single_invoke`` / ``ml_single_set_input_info`` / ``ml_single_set_timeout``
/ ``ml_single_close``; reference gst/nnstreamer/tensor_filter/
tensor_filter_single.c) without building a pipeline.

The native ``SingleShot`` (csrc/single/single.cc) opens the tensor_filter
framework directly; a GPU model stays resident in HBM for the life of the
handle and each invoke runs on the handle's own HIP stream.

    with nns.Single("mobilenet_v2.pt", framework="pytorch",
                    input=[nns.TensorShape([3, 224, 224, 1], np.float32)],
                    accelerator="true:gpu") as s:
        (logits,) = s.invoke(frame)

Inputs are numpy arrays, bytes, ``Memory`` objects or torch tensors (CUDA
tensors are passed zero-copy).  Outputs are numpy arrays shaped from the
output info (NNStreamer dims are innermost-first, numpy shapes the reverse),
or zero-copy torch tensors with ``output="torch"``.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import numpy as np

from . import _C
from .utils.tensors import to_numpy, to_torch

TimeoutError = _C.NnsxTimeout  # noqa: A001  (subclass of the builtin TimeoutError)


def _dtype_name(shape) -> str:
    t = shape.getType()
    return "bfloat16" if str(t) == "bfloat16" else np.dtype(t).name


class Single:
    """One opened model (``ml_single_h``)."""

    def __init__(self, model, framework: str = "auto", input: Optional[Sequence] = None,  # noqa: A002
                 output: Optional[Sequence] = None, accelerator: str = "", custom: str = "",
                 device: int = -1, timeout_ms: int = 0):
        models = [model] if isinstance(model, str) else list(model)
        self._h = _C.SingleShot(framework, models, None if input is None else list(input),
                                None if output is None else list(output), accelerator, custom, device)
        if timeout_ms:
            self._h.set_timeout(int(timeout_ms))

    # ------------------------------------------------------------- info ----
    @property
    def input_info(self) -> List:
        return self._h.input_info()

    @property
    def output_info(self) -> List:
        return self._h.output_info()

    @property
    def framework(self) -> str:
        return self._h.framework()

    @property
    def device(self) -> int:
        """GPU index the model runs on (-1: host)."""
        return self._h.device()

    def set_input_info(self, shapes: Sequence) -> None:
        """Reconfigure for new input dims (the framework reports the new output info)."""
        self._h.set_input_info(list(shapes))

    @property
    def timeout(self) -> int:
        return self._h.timeout()

    @timeout.setter
    def timeout(self, ms: int) -> None:
        self._h.set_timeout(int(ms))

    # ----------------------------------------------------------- invoke ----
    def invoke_dynamic(self, *inputs, output: str = "numpy"):
        """Run once; returns (outputs, output_info) -- the info may change per call."""
        if len(inputs) == 1 and isinstance(inputs[0], (list, tuple)):
            inputs = tuple(inputs[0])
        mems, info = self._h.invoke(list(inputs))
        return [self._convert(m, i, output) for m, i in zip(mems, _pad(info, len(mems)))], info

    def invoke(self, *inputs, output: str = "numpy"):
        """Run once on the given input tensors; returns one array per output tensor."""
        return self.invoke_dynamic(*inputs, output=output)[0]

    @staticmethod
    def _convert(mem, shape, output: str):
        if output == "memory":
            return mem
        if shape is None:
            return mem.numpy("uint8") if output == "numpy" else to_torch(mem, "uint8")
        dims = shape.getDims()
        while len(dims) > 1 and dims[-1] == 1:
            dims = dims[:-1]
        if output == "torch":
            return to_torch(mem, _dtype_name(shape), dims)
        return to_numpy(mem, _dtype_name(shape), dims)

    # ---------------------------------------------------------- closing ----
    def close(self) -> None:
        self._h.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _pad(info, n):
    info = list(info)
    return info + [None] * (n - len(info))
