import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


def _has_gpu():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _has_gpu():
        return
    skip = pytest.mark.skip(reason="no GPU in this environment")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def nns():
    import nnstreamer_amd

    return nnstreamer_amd


@pytest.fixture(scope="session")
def workdir(tmp_path_factory):
    return str(tmp_path_factory.mktemp("nnsx"))


@pytest.fixture(scope="session")
def mbv2_model(workdir):
    from nnstreamer_amd.models.export import export

    return export("mobilenet_v2", os.path.join(workdir, "mbv2_nhwc.pt"), layout="nhwc")


@pytest.fixture(scope="session")
def labels(workdir):
    from nnstreamer_amd.models.export import write_labels

    return write_labels(os.path.join(workdir, "labels.txt"))


def run_pipeline(nns, desc, sink="sink", timeout=60, collect=None):
    """Run a launch string to EOS and return the buffers seen at `sink`."""
    p = nns.parse_launch(desc)
    out = []
    s = p.get_by_name(sink)
    if s is not None:
        s.connect("new-data", (lambda b: out.append(collect(b))) if collect else out.append)
    p.run(timeout=timeout)
    p.stop()
    return out
