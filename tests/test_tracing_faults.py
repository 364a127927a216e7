"""Auxiliary subsystems: built-in tracers, DOT dumps, failure
detection and fault injection."""
import json
import os

import numpy as np
import pytest

F4 = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"


def _run_frames(nns, middle, n=20, timeout=30):
    p = nns.parse_launch(f"appsrc name=src caps={F4} ! {middle} ! tensor_sink name=sink")
    got = []
    p.get_by_name("sink").connect("new-data", lambda b: got.append(float(b.memory(0).numpy("float32")[0])))
    p.set_state("playing")
    src = p.get_by_name("src")
    for i in range(n):
        src.push_buffer(np.full(4, i, np.float32), pts=i)
    src.end_of_stream()
    msg = p.wait(timeout)
    return p, got, msg


def test_tracers_report_every_element(nns):
    nns.tracer_reset()
    nns.tracer_enable("proctime;interlatency;framerate")
    try:
        p, got, msg = _run_frames(nns, "queue ! tensor_transform name=tt mode=arithmetic option=mul:2 "
                                        "! fault_inject name=fi delay-ms=2", n=10)
        p.stop()
    finally:
        nns.tracer_enable("")
    assert msg[0] == "eos" and got == [2.0 * i for i in range(10)]
    rep = json.loads(nns.tracer_report())
    assert set(rep["tracers"]) == set()  # disabled again
    el = rep["elements"]
    for name in ("tt", "fi", "sink"):
        assert el[name]["buffers"] == 10, el
    # the injected 2 ms shows up as fault_inject's processing time and in the sink's interlatency
    assert el["fi"]["proctime_us"]["avg"] >= 1900
    assert el["sink"]["interlatency_us"]["avg"] >= el["tt"]["interlatency_us"]["avg"] + 1900
    assert el["tt"]["fps"] > 0


def test_dot_dump_on_state_change(nns, tmp_path, monkeypatch):
    monkeypatch.setenv("NNSX_DEBUG_DUMP_DOT_DIR", str(tmp_path))
    p = nns.parse_launch("videotestsrc num-buffers=2 ! tensor_converter ! fakesink")
    p.run(timeout=30)
    p.stop()
    files = sorted(os.listdir(tmp_path))
    assert any(f.endswith(".PLAYING.dot") or f.endswith(".playing.dot") for f in files), files
    text = (tmp_path / [f for f in files if "PLAYING" in f.upper()][0]).read_text()
    assert text.startswith("digraph") and "tensor_converter" in text and "->" in text


def test_fault_inject_drop_and_eos(nns):
    p, got, msg = _run_frames(nns, "fault_inject name=fi drop-every=3")
    assert msg[0] == "eos"
    assert got == [float(i) for i in range(20) if (i + 1) % 3 != 0]
    assert p.get_by_name("fi").get_property("dropped") == "6"
    p.stop()
    p, got, msg = _run_frames(nns, "fault_inject eos-after=5")
    assert msg[0] == "eos" and got == [0.0, 1.0, 2.0, 3.0, 4.0]
    p.stop()


@pytest.mark.parametrize("mode", ["fail-after", "throw-after"])
def test_injected_failure_reaches_the_bus(nns, mode):
    """An element error -- or an exception thrown inside chain -- ends the run
    with an error message naming the element instead of a dead thread."""
    p, got, msg = _run_frames(nns, f"queue ! fault_inject name=bad {mode}=3")
    assert msg is not None and msg[0] == "error", p.messages()
    assert msg[1] == "bad" and "injected" in msg[2]
    assert got == [0.0, 1.0, 2.0]
    p.stop()


def test_fault_inject_random_drops_are_seeded(nns):
    a = _run_frames(nns, "fault_inject drop-probability=0.5 seed=7", n=40)
    b = _run_frames(nns, "fault_inject drop-probability=0.5 seed=7", n=40)
    for p, _, _ in (a, b):
        p.stop()
    assert a[1] == b[1] and 5 < len(a[1]) < 35
