"""tensor_filter statistics rules against the reference
(gst/nnstreamer/tensor_filter/tensor_filter.c:378-495, :1314-1376;
tensor_filter_common.c:579):

* the first invoke is ignored (latency_ignore_count = 1);
* `latency` = mean of the last 10 invoke latencies in us;
* `throughput` = invokes x 1e6 x 1000 / total invoke latency (us): FPS x 1000
  of the invoke itself, independent of gaps between frames;
* `latency-report`: a LATENCY message whenever the estimate exceeds what the
  last latency query reported (estimate x 1.05) or deviates from it by > 25 %.

A python3 filter sleeps a scripted time per invoke so every rule is observable.
"""
import time

import numpy as np
import pytest

CAPS = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"


@pytest.fixture()
def sleeper(workdir):
    path = f"{workdir}/sleeper.py"
    with open(path, "w") as f:
        f.write(
            "import time\nimport numpy as np\nimport nnstreamer_python as nns\n"
            "class CustomFilter(object):\n"
            "    def __init__(self, *args):\n"
            "        self.sched = [float(x) for x in args[0].split(':')] if args else [0.0]\n"
            "        self.i = 0\n"
            "    def setInputDim(self, dims):\n        return [nns.TensorShape(dims[0].getDims(), np.float32)]\n"
            "    def invoke(self, arr):\n"
            "        d = self.sched[min(self.i, len(self.sched) - 1)]\n"
            "        self.i += 1\n"
            "        time.sleep(d)\n"
            "        return [arr[0]]\n")
    return path


def _start(nns, sleeper, sched, extra=""):
    p = nns.parse_launch(f"appsrc name=src caps={CAPS} ! tensor_filter name=f framework=python3 model={sleeper} "
                         f"custom={':'.join(str(s) for s in sched)} {extra} ! tensor_sink name=sink")
    got = []
    p.get_by_name("sink").connect("new-data", lambda b: got.append(b))
    p.set_state("playing")
    return p, p.get_by_name("src"), p.get_by_name("f"), got


def _push(src, got, n, gap_s=0.0):
    want = len(got) + n
    for _ in range(n):
        src.push_buffer(np.zeros(4, np.float32))
        if gap_s:
            time.sleep(gap_s)
    t = time.time()
    while len(got) < want and time.time() - t < 20:
        time.sleep(0.005)
    assert len(got) == want


def test_first_invoke_ignored_and_recent_mean(nns, sleeper):
    # invoke 0 takes 150 ms (ignored), the next 5 take 5 ms
    p, src, f, got = _start(nns, sleeper, [0.15, 0.005], "latency=1 throughput=1")
    _push(src, got, 6)
    lat = f.get_property("latency")
    src.end_of_stream()
    p.wait(timeout=10)
    p.stop()
    assert 4000 <= lat < 20000, lat  # with the 150 ms sample included the mean would be >= 29 ms


def test_throughput_is_invoke_rate_not_arrival_rate(nns, sleeper):
    # 5 ms invokes, frames 60 ms apart: the reference reports ~200 FPS (x1000), not ~16
    p, src, f, got = _start(nns, sleeper, [0.005], "latency=1 throughput=1")
    _push(src, got, 6, gap_s=0.06)
    thr = f.get_property("throughput")
    src.end_of_stream()
    p.wait(timeout=10)
    p.stop()
    assert 100_000 <= thr <= 210_000, thr


def test_stats_disabled_read_minus_one(nns, sleeper):
    p, src, f, got = _start(nns, sleeper, [0.0])
    _push(src, got, 3)
    assert f.get_property("latency") == -1 and f.get_property("throughput") == -1
    src.end_of_stream()
    p.wait(timeout=10)
    p.stop()


def test_latency_report_rules(nns, sleeper):
    # 50 ms for 8 invokes, then 150 ms (long enough that sleep overshoot on a
    # loaded host -- a few ms per invoke -- stays inside the 5 % headroom)
    p, src, f, got = _start(nns, sleeper, [0.05] * 9 + [0.15], "latency-report=true")
    sink = p.get_by_name("sink")

    def posts():
        return sum(1 for m in p.messages() if m[0] == "latency" and m[1] == "f")

    _push(src, got, 3)  # first sample ignored; then estimate > reported (0): posted
    assert posts() >= 1
    q = sink.query_latency()  # reported := estimate x 1.05, added to the pipeline latency
    assert q is not None and q[1] >= 48_000_000, q
    _push(src, got, 4)  # steady 50 ms: inside the headroom, within 25 %: nothing posted
    assert posts() == 0
    _push(src, got, 3)  # 150 ms invokes: estimate above the reported value: posted again
    assert posts() >= 1
    src.end_of_stream()
    p.wait(timeout=10)
    p.stop()
