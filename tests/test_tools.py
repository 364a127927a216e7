"""nnsx-check / nnsx-launch command-line tools (reference confchk and gst-launch):
the native executables bin/nnsx-check and bin/nnsx-launch (csrc/tools), plus
the Python modules of the same names."""
import json

import numpy as np
import pytest
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, NNSX_DISABLE_GPU="1")


def _run(*args, timeout=120):
    return subprocess.run([sys.executable, "-m", *args], cwd=ROOT, env=ENV, capture_output=True, text=True,
                          timeout=timeout)


def _native(tool, *args, timeout=120):
    return subprocess.run([os.path.join(ROOT, "bin", tool), *args], cwd=ROOT, env=ENV, capture_output=True, text=True,
                          timeout=timeout)


def test_native_check_json():
    r = _native("nnsx-check", "--json")
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert "tensor_filter" in d["elements"] and "pytorch" in d["subplugins"]["filter"]
    assert "bounding_boxes" in d["subplugins"]["decoder"] and d["version"].startswith("nnsx")


def test_native_launch_eos_caps_and_errors(tmp_path):
    dot = tmp_path / "g.dot"
    r = _native("nnsx-launch", "-v", "--dot", str(dot), "videotestsrc", "num-buffers=3", "!",
                "video/x-raw,format=RGB,width=8,height=4", "!", "tensor_converter", "!", "tensor_sink")
    assert r.returncode == 0, r.stderr
    assert "dimensions=(string)3:8:4:1" in r.stdout and "Got EOS" in r.stdout
    assert "digraph" in dot.read_text()
    assert _native("nnsx-launch", "nosuchelement ! fakesink").returncode == 2
    assert _native("nnsx-launch", "-t", "1", "videotestsrc is-live=true ! fakesink").returncode == 3
    r = _native("nnsx-launch", "-m", "videotestsrc num-buffers=2 ! tensor_converter ! tensor_sink")
    assert r.returncode == 0 and "Got message from" in r.stdout


def test_check_json():
    r = _run("nnstreamer_amd.tools.check", "--json")
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert "tensor_filter" in d["elements"] and "pytorch" in d["subplugins"]["filter"]
    assert "bounding_boxes" in d["subplugins"]["decoder"]


def test_launch_eos_and_caps(tmp_path):
    dot = tmp_path / "g.dot"
    r = _run("nnstreamer_amd.tools.launch", "-v", "--dot", str(dot),
             "videotestsrc num-buffers=3 ! video/x-raw,format=RGB,width=8,height=4 ! tensor_converter ! tensor_sink")
    assert r.returncode == 0, r.stderr
    assert "dimensions=(string)3:8:4:1" in r.stdout and "Got EOS" in r.stdout
    assert "digraph" in dot.read_text()


def test_launch_errors():
    assert _run("nnstreamer_amd.tools.launch", "nosuchelement ! fakesink").returncode == 2
    r = _run("nnstreamer_amd.tools.launch", "-t", "1", "videotestsrc is-live=true ! fakesink")
    assert r.returncode == 3


def test_pbtxt_matches_reference_converter_naming(nns):
    """convert.c naming: sources/sinks are graph streams, internal streams
    <factory>_<index>_<srcpad>, repeated factories <factory>_<n>."""
    p = nns.parse_launch("videotestsrc num-buffers=1 ! video/x-raw,format=RGB,width=8,height=8 ! tensor_converter "
                         "! tee name=t t. ! queue ! tensor_sink t. ! queue ! fakesink")
    txt = nns.to_pbtxt(p)
    assert txt.startswith('input_stream: "videotestsrc"\noutput_stream: "tensor_sink"\noutput_stream: "fakesink"\n')
    assert 'calculator: "teeCalculator"\n\tinput_stream: "tensor_converter_0_0"\n\toutput_stream: "tee_0_0"\n' \
           '\toutput_stream: "tee_0_1"' in txt
    assert txt.count('calculator: "queueCalculator"') == 2
    assert "capsfilter" not in txt  # caps are link attributes


def test_pbtxt_roundtrip_runs(nns):
    desc = ("videotestsrc num-buffers=3 ! video/x-raw,format=RGB,width=8,height=8 ! tensor_converter "
            "! tensor_transform mode=typecast option=float32 ! tensor_sink name=out")
    txt = nns.to_pbtxt(nns.parse_launch(desc), True)
    back = nns.pbtxt_to_launch(txt)
    p = nns.parse_launch(back)
    got = []
    p.get_by_name("tensor_sink").connect("new-data", lambda b: got.append(b.memory(0).size))
    p.run(timeout=30)
    p.stop()
    assert got == [8 * 8 * 3 * 4] * 3


def test_pbtxt_cli(tmp_path):
    import subprocess
    import sys
    out = subprocess.run([sys.executable, "-m", "nnstreamer_amd.tools.pbtxt", "videotestsrc ! tensor_converter ! fakesink"],
                         capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert out.returncode == 0, out.stderr
    assert 'calculator: "tensor_converterCalculator"' in out.stdout
    bad = subprocess.run([sys.executable, "-m", "nnstreamer_amd.tools.pbtxt", "-p"], input="node: { input_stream: \"x\" }",
                         capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert bad.returncode == 1 and "calculator" in bad.stderr


@pytest.mark.parametrize("dynamic,allocate", [(False, False), (True, True)])
def test_codegen_c_skeleton_builds_and_runs(nns, tmp_path, dynamic, allocate):
    from nnstreamer_amd.tools.codegen import generate
    files = generate("My Filter", dynamic, allocate, "c", str(tmp_path))
    r = subprocess.run(["sh", files[1]], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lib = tmp_path / "libnnsx_customfilter_my_filter.so"
    caps = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_filter framework=custom model={lib} ! tensor_sink name=s")
    got = []
    p.get_by_name("s").connect("new-data", lambda b: got.append(b.memory(0).numpy("float32").copy()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(np.arange(4, dtype=np.float32), pts=0)
    p.get_by_name("src").end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    p.stop()
    np.testing.assert_array_equal(got[0], np.arange(4, dtype=np.float32))


def test_codegen_python_skeleton_runs(nns, tmp_path):
    from nnstreamer_amd.tools.codegen import generate
    path = generate("py filter", False, False, "python", str(tmp_path))[0]
    caps = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_filter framework=python3 model={path} ! tensor_sink name=s")
    got = []
    p.get_by_name("s").connect("new-data", lambda b: got.append(b.memory(0).numpy("float32").copy()))
    p.set_state("playing")
    p.get_by_name("src").push_buffer(np.ones(4, dtype=np.float32), pts=0)
    p.get_by_name("src").end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    p.stop()
    np.testing.assert_array_equal(got[0], np.ones(4, dtype=np.float32))


def test_parallel_helpers(monkeypatch):
    import nnstreamer_amd.parallel as P
    monkeypatch.setenv("RANK", "2")
    monkeypatch.setenv("WORLD_SIZE", "3")
    monkeypatch.setenv("LOCAL_RANK", "2")
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("MASTER_PORT", "30000")
    monkeypatch.delenv("NNSX_STORE", raising=False)
    info = P.rank_info(use_gpu=False)
    assert (info.rank, info.world, info.device, info.store) == (2, 3, -1, "127.0.0.1:30017")
    assert list(P.split_work(10, info)) == [7, 8, 9]
    assert P.format_pipeline("tensor_allgather rank={rank} store={store}", info) == \
        "tensor_allgather rank=2 store=127.0.0.1:30017"
    assert P.gather_stats([1.5]) == [1.5]  # no process group: identity


@pytest.mark.skipif(os.environ.get("NNSX_TSAN") != "1", reason="ThreadSanitizer build takes ~2 min: NNSX_TSAN=1")
def test_tsan_host_runtime():
    """scripts/tsan_check.sh: TSan build of the host runtime driving the threaded
    elements (queue/tee/mux, query server+clients, MQTT, rank groups); exit 66 = race."""
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "tsan_check.sh")], capture_output=True, text=True,
                       timeout=1500)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr
