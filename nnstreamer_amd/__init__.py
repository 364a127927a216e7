"""nnstreamer_amd -- an MI355X-native neural-network streaming framework with
NNStreamer's element set (tensor_converter, tensor_transform, tensor_filter,
tensor_decoder, tensor_mux/demux/merge/split, ...) and `other/tensors` caps.

The runtime is native C++ (``csrc/``) with hand-written CDNA4 HIP kernels;
this package exposes it to Python::

    import nnstreamer_amd as nns
    p = nns.parse_launch("videotestsrc num-buffers=10 ! tensor_converter ! "
                         "tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 ! "
                         "tensor_sink name=s")
    p.get_by_name("s").connect("new-data", lambda buf: ...)
    p.run()
"""
from __future__ import annotations

import os
import sys

# torch first: its bundled HIP runtime (libamdhip64.so.7) must be the one our
# extension binds to (same SONAME -> one runtime per process).
import torch  # noqa: F401

_here = os.path.dirname(os.path.abspath(__file__))
_root = os.path.dirname(_here)
if _root not in sys.path:
    sys.path.insert(0, _root)  # makes `import nnstreamer_python` work for user scripts


def _load():
    try:
        from . import _C  # noqa: F401
    except ImportError as e:  # pragma: no cover - exercised when the .so is missing
        if os.environ.get("NNSX_AUTOBUILD", "1") != "0":
            from . import _build

            _build.build()
            from . import _C  # noqa: F401,F811
        else:
            raise ImportError(f"nnstreamer_amd native extension is not built: {e}") from e
    return _C


_C = _load()

from ._C import (  # noqa: E402,F401
    Buffer,
    Caps,
    Element,
    Group,
    Memory,
    MqttBroker,
    Packet,
    NnsxError,
    Pipeline,
    config_dump,
    config_value,
    dimension_string,
    dimension_string_equal,
    dtype_from_string,
    dtype_name,
    dtype_size,
    element_exists,
    bind_numa,
    gpu_arch,
    gpu_count,
    gpu_numa_node,
    kernels,
    last_error,
    list_elements,
    load_subplugin_library,
    make_element,
    memory_from,
    meta_header,
    parse_dimension,
    parse_launch,
    parse_meta_header,
    pbtxt_to_launch,
    to_pbtxt,
    tracer_enable,
    tracer_report,
    tracer_reset,
    register_converter_custom,
    register_custom_easy,
    register_decoder_custom,
    register_if_custom,
    set_debug,
    subplugins,
    unregister_converter_custom,
    unregister_custom_easy,
    unregister_decoder_custom,
    unregister_if_custom,
    version,
)
from .utils.tensors import TensorShape, to_numpy, to_torch  # noqa: E402,F401
from .single import Single  # noqa: E402,F401

__all__ = [
    "Buffer",
    "Caps",
    "Element",
    "Group",
    "Packet",
    "Memory",
    "Pipeline",
    "TensorShape",
    "Single",
    "parse_launch",
    "make_element",
    "to_numpy",
    "to_torch",
    "version",
]
