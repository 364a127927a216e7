"""`import nnstreamer_python as nns` -- the module the reference's Python
filter/converter/decoder scripts import (TensorShape).  Provided by
nnstreamer_amd so such scripts run unchanged."""
from nnstreamer_amd.utils.tensors import TensorShape  # noqa: F401
