"""Among-device elements over TCP (reference: tests/nnstreamer_edge/query/
runTest.sh and edge/runTest.sh -- server / publisher pipelines in the
background, clients / subscribers in the foreground).  Both in-process and
separate-process topologies are covered."""
import os
import subprocess
import sys
import textwrap
import time

import numpy as np
import pytest

F32 = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _wait_port(elem, timeout=10):
    t0 = time.time()
    while time.time() - t0 < timeout:
        port = int(elem.get_property("port"))
        if port:
            return port
        time.sleep(0.01)
    raise AssertionError("server did not bind")


def _register_double(nns):
    nns.register_custom_easy("comm_double", lambda x: [x[0] * 2],
                             [nns.TensorShape([4], np.float32)], [nns.TensorShape([4], np.float32)])


def _client_run(nns, port, frames, extra=""):
    p = nns.parse_launch(f"appsrc name=src caps={F32} ! tensor_query_client dest-host=127.0.0.1 dest-port={port} "
                         f"{extra} ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append((b.pts, b.memory(0).numpy("float32").copy())))
    p.set_state("playing")
    for i, f in enumerate(frames):
        p.get_by_name("src").push_buffer(f, pts=1000 + i)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(30)
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    return out


def test_query_roundtrip_in_process(nns):
    _register_double(nns)
    server = nns.parse_launch(f"tensor_query_serversrc name=qs id=11 port=0 ! {F32} "
                              "! tensor_filter framework=custom-easy model=comm_double ! tensor_query_serversink id=11")
    server.set_state("playing")
    port = _wait_port(server.get_by_name("qs"))
    frames = [np.arange(4, dtype=np.float32) + i for i in range(5)]
    out = _client_run(nns, port, frames)
    assert [t for t, _ in out] == [1000 + i for i in range(5)]
    for (_, y), x in zip(out, frames):
        np.testing.assert_array_equal(y, 2 * x)
    # pipelined requests (max-request) keep order
    out = _client_run(nns, port, frames, "max-request=3")
    for (_, y), x in zip(out, frames):
        np.testing.assert_array_equal(y, 2 * x)
    server.stop()


def test_query_two_clients_routed_by_id(nns):
    _register_double(nns)
    server = nns.parse_launch(f"tensor_query_serversrc name=qs id=12 port=0 ! {F32} "
                              "! tensor_filter framework=custom-easy model=comm_double ! tensor_query_serversink id=12")
    server.set_state("playing")
    port = _wait_port(server.get_by_name("qs"))
    import threading
    res = {}

    def run(k):
        res[k] = _client_run(nns, port, [np.full(4, k * 10 + i, np.float32) for i in range(20)])

    th = [threading.Thread(target=run, args=(k,)) for k in (1, 2)]
    [t.start() for t in th]
    [t.join() for t in th]
    server.stop()
    for k in (1, 2):
        assert [float(y[0]) for _, y in res[k]] == [2.0 * (k * 10 + i) for i in range(20)]


def test_query_server_in_other_process(nns, tmp_path):
    script = tmp_path / "server.py"
    script.write_text(textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import numpy as np
        import nnstreamer_amd as nns
        nns.register_custom_easy("neg", lambda x: [-x[0]], [nns.TensorShape([4], np.float32)],
                                 [nns.TensorShape([4], np.float32)])
        p = nns.parse_launch("tensor_query_serversrc name=qs port=0 ! {F32} "
                             "! tensor_filter framework=custom-easy model=neg ! tensor_query_serversink")
        p.set_state("playing")
        while int(p.get_by_name("qs").get_property("port")) == 0:
            time.sleep(0.01)
        print(p.get_by_name("qs").get_property("port"), flush=True)
        sys.stdin.readline()
        p.stop()
    """))
    proc = subprocess.Popen([sys.executable, str(script)], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        port = int(proc.stdout.readline())
        out = _client_run(nns, port, [np.arange(4, dtype=np.float32)])
        np.testing.assert_array_equal(out[0][1], -np.arange(4, dtype=np.float32))
    finally:
        proc.stdin.write("\n")
        proc.stdin.flush()
        proc.wait(timeout=30)


def test_query_client_errors_without_server(nns):
    p = nns.parse_launch(f"appsrc name=src caps={F32} ! tensor_query_client dest-port=1 timeout=300 ! tensor_sink name=sink")
    with pytest.raises(Exception):
        p.set_state("playing")
        msg = p.wait(15)
        assert msg is None or msg[0] == "error"
        raise RuntimeError("no server")
    p.stop()


def test_edge_pubsub_two_subscribers(nns):
    pub = nns.parse_launch(f"appsrc name=src caps={F32} ! edgesink name=es port=0 wait-connection=2")
    pub.set_state("playing")
    port = _wait_port(pub.get_by_name("es"))
    subs, outs = [], []
    for k in range(2):
        s = nns.parse_launch(f"edgesrc dest-host=127.0.0.1 dest-port={port} ! tensor_sink name=sink")
        o = []
        s.get_by_name("sink").connect("new-data", lambda b, o=o: o.append(b.memory(0).numpy("float32").copy()))
        s.set_state("playing")
        subs.append(s)
        outs.append(o)
    frames = [np.full(4, i, np.float32) for i in range(6)]
    for i, f in enumerate(frames):
        pub.get_by_name("src").push_buffer(f, pts=i)
    pub.get_by_name("src").end_of_stream()
    assert pub.wait(20)[0] == "eos"
    for s, o in zip(subs, outs):
        msg = s.wait(20)
        assert msg and msg[0] == "eos", s.messages()
        s.stop()
        assert [float(x[0]) for x in o] == [float(i) for i in range(6)]
    pub.stop()


def test_edge_shm_frames_by_reference_across_processes(nns, tmp_path):
    """connect-type=SHM: the publisher's camera ring lives in a POSIX shared
    segment (videotestsrc pool-shm); frames reach a subscriber in ANOTHER
    process as references into that segment (zero-copy: shm-blobs counts them),
    byte-identical to the camera's, and every frame is handed back (the
    publisher's pipeline finishes).  On a GPU the subscriber's mapping is
    hipHostRegister'ed, so its own tensor_converter DMAs the frames over its
    GPU's link (tests/test_gpu_shm_ingest.py).  Reference fan-out this
    replaces across processes: gsttensor_demux.c:469-556 (buffers by reference)."""
    import os

    name = f"nnsx-test-{os.getpid()}"
    script = tmp_path / "pub.py"
    script.write_text(textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import nnstreamer_amd as nns
        p = nns.parse_launch("videotestsrc num-buffers=24 pattern=snow pool-size=6 pool-shm={name} "
                             "! video/x-raw,format=RGB,width=64,height=48,framerate=0/1 "
                             "! edgesink name=es port=0 connect-type=SHM wait-connection=1")
        p.set_state("playing")
        while int(p.get_by_name("es").get_property("port")) == 0:
            time.sleep(0.01)
        print(p.get_by_name("es").get_property("port"), flush=True)
        msg = p.wait(60)
        print(msg[0] if msg else "timeout", flush=True)
        sys.stdin.readline()
        p.stop()
    """))
    proc = subprocess.Popen([sys.executable, str(script)], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True)
    try:
        port = int(proc.stdout.readline())
        s = nns.parse_launch(f"edgesrc name=src dest-host=127.0.0.1 dest-port={port} connect-type=SHM "
                             "! tensor_converter ! tensor_sink name=sink")
        out = []
        s.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).numpy("uint8").copy()))
        s.set_state("playing")
        msg = s.wait(60)
        assert msg and msg[0] == "eos", s.messages()
        shm_blobs = int(s.get_by_name("src").get_property("shm-blobs"))
        s.stop()
        assert proc.stdout.readline().strip() == "eos"
    finally:
        proc.stdin.write("\n")
        proc.stdin.flush()
        proc.wait(timeout=30)
    assert len(out) == 24 and shm_blobs == 24, (len(out), shm_blobs)
    # the camera's snow frames, in ring order (pool of 6 distinct frames)
    ref = nns.parse_launch("videotestsrc num-buffers=6 pattern=snow pool-size=6 "
                           "! video/x-raw,format=RGB,width=64,height=48,framerate=0/1 ! tensor_converter "
                           "! tensor_sink name=sink")
    want = []
    ref.get_by_name("sink").connect("new-data", lambda b: want.append(b.memory(0).numpy("uint8").copy()))
    ref.run(timeout=30)
    for i, fr in enumerate(out):
        np.testing.assert_array_equal(fr.ravel(), want[i % 6].ravel())
