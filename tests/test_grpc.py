"""tensor_src_grpc / tensor_sink_grpc (reference tests/nnstreamer_grpc/runTest.sh:
sink-client -> src-server and sink-server -> src-client, protobuf and flatbuf IDLs)."""
import time

import numpy as np
import pytest

pytest.importorskip("grpc")

CAPS = "other/tensors,format=static,num_tensors=1,dimensions=3:16:8:1,types=uint8,framerate=30/1"
SRC = "videotestsrc num-buffers={n} pattern=snow ! video/x-raw,format=RGB,width=16,height=8,framerate=30/1 ! tensor_converter"


def _frames(nns, n):
    p = nns.parse_launch(SRC.format(n=n) + " ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes()))
    p.run(timeout=30)
    return out


def _wait_port(e):
    t0 = time.time()
    while time.time() - t0 < 10:
        port = int(e.get_property("port"))
        if port:
            return port
        time.sleep(0.01)
    raise AssertionError("no port")


@pytest.mark.parametrize("idl", ["protobuf", "flatbuf"])
def test_sink_client_to_src_server(nns, idl):
    expected = _frames(nns, 5)
    srv = nns.parse_launch(f"tensor_src_grpc name=gs server=true port=0 idl={idl} ! {CAPS} ! tensor_sink name=sink")
    got = []
    srv.get_by_name("sink").connect("new-data", lambda b: got.append(b.memory(0).bytes()))
    srv.set_state("playing")
    port = _wait_port(srv.get_by_name("gs"))
    cli = nns.parse_launch(SRC.format(n=5) + f" ! tensor_sink_grpc name=gk host=127.0.0.1 port={port} idl={idl}")
    cli.run(timeout=30)
    assert int(cli.get_by_name("gk").get_property("out")) == 5
    t0 = time.time()
    while len(got) < 5 and time.time() - t0 < 10:
        time.sleep(0.02)
    srv.stop()
    assert got == expected


@pytest.mark.parametrize("idl", ["protobuf", "flatbuf"])
def test_sink_server_to_src_client(nns, idl):
    pub = nns.parse_launch(f"appsrc name=src caps={CAPS} ! tensor_sink_grpc name=gk server=true port=0 idl={idl}")
    pub.set_state("playing")
    port = _wait_port(pub.get_by_name("gk"))
    sub = nns.parse_launch(f"tensor_src_grpc name=gs server=false host=127.0.0.1 port={port} idl={idl} "
                           f"! {CAPS} ! tensor_sink name=sink")
    got = []
    sub.get_by_name("sink").connect("new-data", lambda b: got.append((b.pts, b.memory(0).bytes())))
    sub.set_state("playing")
    time.sleep(1.0)  # the RecvTensors call is in place before publishing
    frames = [np.full(3 * 16 * 8, i, np.uint8) for i in range(4)]
    for i, f in enumerate(frames):
        pub.get_by_name("src").push_buffer(f, pts=i)
    pub.get_by_name("src").end_of_stream()
    assert pub.wait(20)[0] == "eos"
    pub.stop()  # ends the server streams -> the client source reaches EOS
    msg = sub.wait(20)
    sub.stop()
    assert msg and msg[0] == "eos", sub.messages()
    assert [b for _, b in got] == [f.tobytes() for f in frames]
    # timestamps from the negotiated framerate (30/1)
    assert [t for t, _ in got] == [i * 1_000_000_000 // 30 for i in range(4)]


def test_client_without_server_errors(nns):
    p = nns.parse_launch(SRC.format(n=1) + " ! tensor_sink_grpc host=127.0.0.1 port=1")
    with pytest.raises(Exception):
        p.set_state("playing")
        msg = p.wait(20)
        assert msg is None or msg[0] == "error"
        raise RuntimeError("expected")
    p.stop()
