"""Native HTTP/2 gRPC transport (csrc/comm/grpc_native.cc, csrc/comm/hpack.cc):
HPACK against the RFC 7541 Appendix C vectors, and wire interop of
tensor_sink_grpc / tensor_src_grpc with grpcio peers (the role the reference's
grpc++ plays: ext/nnstreamer/extra/nnstreamer_grpc_common.cc:83-200), all four
directions of TensorService plus an unserved method."""
import queue
import threading
import time
from concurrent import futures

import numpy as np
import pytest

from nnstreamer_amd import _C

grpc = pytest.importorskip("grpc")

CAPS = "other/tensors,format=static,num_tensors=1,dimensions=3:16:8:1,types=uint8,framerate=30/1"
SERVICE = "nnstreamer.protobuf.TensorService"


# ----------------------------------------------------------------- HPACK ----
@pytest.mark.parametrize("text,hexcode", [
    ("www.example.com", "f1e3c2e5f23a6ba0ab90f4ff"), ("no-cache", "a8eb10649cbf"),
    ("custom-key", "25a849e95ba97d7f"), ("custom-value", "25a849e95bb8e8b4bf"), ("302", "6402"),
    ("private", "aec3771a4b"), ("Mon, 21 Oct 2013 20:13:21 GMT", "d07abe941054d444a8200595040b8166e082a62d1bff"),
    ("https://www.example.com", "9d29ad171863c78f0b97c8e9ae82ae43d3"), ("gzip", "9bd9ab")])
def test_huffman_rfc7541_vectors(text, hexcode):
    assert _C.hpack_huffman_encode(text).hex() == hexcode
    assert _C.hpack_huffman_decode(bytes.fromhex(hexcode)) == text


def test_huffman_roundtrip_all_bytes_and_bad_padding():
    s = bytes(range(256)).decode("latin-1")
    enc = _C.hpack_huffman_encode(s)
    assert _C.hpack_huffman_decode(enc).encode("latin-1") == bytes(range(256))
    with pytest.raises(ValueError):
        _C.hpack_huffman_decode(bytes.fromhex("f1e3c2e5f23a6ba0ab90f4fe"))  # padding not all ones


REQ = [(":method", "GET"), (":scheme", "http"), (":path", "/"), (":authority", "www.example.com")]


@pytest.mark.parametrize("blocks", [
    # C.3: requests without Huffman coding
    ["828684410f7777772e6578616d706c652e636f6d", "828684be58086e6f2d6361636865",
     "828785bf400a637573746f6d2d6b65790c637573746f6d2d76616c7565"],
    # C.4: the same requests with Huffman coding
    ["828684418cf1e3c2e5f23a6ba0ab90f4ff", "828684be5886a8eb10649cbf",
     "828785bf408825a849e95ba97d7f8925a849e95bb8e8b4bf"]])
def test_hpack_decoder_rfc7541_requests(blocks):
    out = _C.hpack_decode_blocks([bytes.fromhex(b) for b in blocks])
    assert [tuple(h) for h in out[0]] == REQ
    assert [tuple(h) for h in out[1]] == REQ + [("cache-control", "no-cache")]
    assert [tuple(h) for h in out[2]] == [(":method", "GET"), (":scheme", "https"), (":path", "/index.html"),
                                          (":authority", "www.example.com"), ("custom-key", "custom-value")]


# ----------------------------------------------------------- grpcio interop --
def _ident(b):
    return b


def _frames(n):
    return [np.full(3 * 16 * 8, 10 + i, np.uint8).tobytes() for i in range(n)]


def _push(nns, pipe_tail, frames):
    p = nns.parse_launch(f"appsrc name=src caps={CAPS} ! {pipe_tail}")
    p.set_state("playing")
    for i, f in enumerate(frames):
        p.get_by_name("src").push_buffer(np.frombuffer(f, np.uint8), pts=i)
    p.get_by_name("src").end_of_stream()
    return p


def _wait_port(e):
    t0 = time.time()
    while time.time() - t0 < 10:
        port = int(e.get_property("port"))
        if port:
            return port
        time.sleep(0.01)
    raise AssertionError("no port")


class _Server:
    """grpcio TensorService on raw bytes: records SendTensors messages,
    streams `to_send` on RecvTensors."""

    def __init__(self, to_send=()):
        self.got, self.to_send = [], list(to_send)
        self.done = threading.Event()
        self.srv = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        handlers = {
            "SendTensors": grpc.stream_unary_rpc_method_handler(self._send, request_deserializer=_ident,
                                                                response_serializer=_ident),
            "RecvTensors": grpc.unary_stream_rpc_method_handler(self._recv, request_deserializer=_ident,
                                                                response_serializer=_ident),
        }
        self.srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(SERVICE, handlers),))
        self.port = self.srv.add_insecure_port("127.0.0.1:0")
        self.srv.start()

    def _send(self, it, ctx):
        for m in it:
            self.got.append(m)
        self.done.set()
        return b""

    def _recv(self, req, ctx):
        assert req == b""
        yield from self.to_send

    def stop(self):
        self.srv.stop(grace=0.5)


def _messages_via_native(nns, frames):
    """Tensors messages as the native sink client sends them (captured by grpcio)."""
    s = _Server()
    try:
        p = _push(nns, f"tensor_sink_grpc host=127.0.0.1 port={s.port}", frames)
        assert p.wait(20)[0] == "eos", p.messages()
        p.stop()
        assert s.done.wait(10)
        return list(s.got)
    finally:
        s.stop()


def test_native_sink_client_to_grpcio_server(nns):
    frames = _frames(5)
    msgs = _messages_via_native(nns, frames)
    assert len(msgs) == 5
    for m, f in zip(msgs, frames):
        assert f in m  # the tensor bytes travel as the protobuf Tensor payload


def test_grpcio_client_to_native_src_server(nns):
    frames = _frames(4)
    msgs = _messages_via_native(nns, frames)
    srv = nns.parse_launch(f"tensor_src_grpc name=gs server=true port=0 ! {CAPS} ! tensor_sink name=sink")
    got = []
    srv.get_by_name("sink").connect("new-data", lambda b: got.append(b.memory(0).bytes()))
    srv.set_state("playing")
    port = _wait_port(srv.get_by_name("gs"))
    with grpc.insecure_channel(f"127.0.0.1:{port}") as ch:
        call = ch.stream_unary(f"/{SERVICE}/SendTensors", request_serializer=_ident, response_deserializer=_ident)
        assert call(iter(msgs), timeout=10) == b""  # google.protobuf.Empty
        # an unserved method: UNIMPLEMENTED
        bad = ch.unary_stream(f"/{SERVICE}/RecvTensors", request_serializer=_ident, response_deserializer=_ident)
        with pytest.raises(grpc.RpcError) as e:
            list(bad(b"", timeout=10))
        assert e.value.code() == grpc.StatusCode.UNIMPLEMENTED
    t0 = time.time()
    while len(got) < 4 and time.time() - t0 < 10:
        time.sleep(0.02)
    srv.stop()
    assert got == frames


def test_native_sink_server_to_grpcio_client(nns):
    frames = _frames(3)
    p = nns.parse_launch(f"appsrc name=src caps={CAPS} ! tensor_sink_grpc name=gk server=true port=0")
    p.set_state("playing")
    port = _wait_port(p.get_by_name("gk"))
    q: "queue.Queue" = queue.Queue()

    def reader():
        with grpc.insecure_channel(f"127.0.0.1:{port}") as ch:
            call = ch.unary_stream(f"/{SERVICE}/RecvTensors", request_serializer=_ident, response_deserializer=_ident)
            try:
                for m in call(b"", timeout=30):
                    q.put(m)
                q.put("end")
            except grpc.RpcError as e:
                q.put(e)

    t = threading.Thread(target=reader)
    t.start()
    t0 = time.time()
    while int(p.get_by_name("gk").get_property("out")) == 0 and time.time() - t0 < 1.0:
        time.sleep(0.05)
    time.sleep(0.5)  # the call is subscribed before the first buffer
    for i, f in enumerate(frames):
        p.get_by_name("src").push_buffer(np.frombuffer(f, np.uint8), pts=i)
    p.get_by_name("src").end_of_stream()
    assert p.wait(20)[0] == "eos"
    p.stop()  # ends the RecvTensors stream with status OK
    t.join(30)
    got = [q.get_nowait() for _ in range(q.qsize())]
    assert got[-1] == "end", got[-1]
    assert len(got) == 4 and all(f in m for f, m in zip(frames, got[:3]))


def test_native_src_client_from_grpcio_server(nns):
    frames = _frames(3)
    s = _Server(to_send=_messages_via_native(nns, frames))
    try:
        sub = nns.parse_launch(f"tensor_src_grpc server=false host=127.0.0.1 port={s.port} ! {CAPS} "
                               "! tensor_sink name=sink")
        got = []
        sub.get_by_name("sink").connect("new-data", lambda b: got.append(b.memory(0).bytes()))
        sub.set_state("playing")
        msg = sub.wait(20)
        sub.stop()
        assert msg and msg[0] == "eos", sub.messages()
        assert got == frames
    finally:
        s.stop()


def test_large_messages_respect_flow_control(nns):
    """Tensors of 3 MB (> the 64 KB default HTTP/2 windows) both ways."""
    caps = "other/tensors,format=static,num_tensors=1,dimensions=3:1024:1024:1,types=uint8,framerate=0/1"
    frames = [np.random.default_rng(i).integers(0, 256, 3 << 20, dtype=np.uint8).tobytes() for i in range(3)]
    srv = nns.parse_launch(f"tensor_src_grpc name=gs server=true port=0 ! {caps} ! tensor_sink name=sink")
    got = []
    srv.get_by_name("sink").connect("new-data", lambda b: got.append(b.memory(0).bytes()))
    srv.set_state("playing")
    port = _wait_port(srv.get_by_name("gs"))
    p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_sink_grpc host=127.0.0.1 port={port}")
    p.set_state("playing")
    for i, f in enumerate(frames):
        p.get_by_name("src").push_buffer(np.frombuffer(f, np.uint8), pts=i)
    p.get_by_name("src").end_of_stream()
    assert p.wait(30)[0] == "eos", p.messages()
    p.stop()
    t0 = time.time()
    while len(got) < 3 and time.time() - t0 < 20:
        time.sleep(0.02)
    srv.stop()
    assert got == frames


# ------------------------------------------------------------- ADVICE r2 ----
FB_SERVICE = "nnstreamer.flatbuf.TensorService"
# flatbuffers FlatBufferBuilder: CreateEmpty(b) + b.Finish() for a table with no
# fields (root uoffset 8 | vtable {size 4, object 4} | soffset 4) -- the message the
# reference's flatbuf peers send and verify (nnstreamer_grpc_flatbuf.cc:269-276,397-402)
FB_EMPTY = bytes.fromhex("08000000" "04000400" "04000000")


def test_flatbuf_empty_request_bytes(nns):
    """idl=flatbuf RecvTensors client sends a finished empty flatbuffer, not 0 bytes."""
    got = []
    done = threading.Event()

    def recv(req, ctx):
        got.append(req)
        done.set()
        return iter(())

    srv = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
    srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(FB_SERVICE, {
        "RecvTensors": grpc.unary_stream_rpc_method_handler(recv, request_deserializer=_ident,
                                                            response_serializer=_ident)}),))
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    try:
        p = nns.parse_launch(f"tensor_src_grpc idl=flatbuf server=false host=127.0.0.1 port={port} ! {CAPS} "
                             "! tensor_sink name=sink")
        p.set_state("playing")
        assert done.wait(10)
        p.wait(10)
        p.stop()
    finally:
        srv.stop(grace=0.2)
    assert got == [FB_EMPTY]


def test_flatbuf_empty_reply_bytes(nns):
    """idl=flatbuf SendTensors server replies with the finished empty flatbuffer."""
    srv = nns.parse_launch(f"tensor_src_grpc name=gs idl=flatbuf server=true port=0 ! {CAPS} ! fakesink")
    srv.set_state("playing")
    port = _wait_port(srv.get_by_name("gs"))
    try:
        with grpc.insecure_channel(f"127.0.0.1:{port}") as ch:
            call = ch.stream_unary(f"/{FB_SERVICE}/SendTensors", request_serializer=_ident,
                                   response_deserializer=_ident)
            assert call(iter(()), timeout=10) == FB_EMPTY
    finally:
        srv.stop()


def test_oversize_message_resource_exhausted(nns):
    """A message above max-recv-message-size ends the call with RESOURCE_EXHAUSTED
    before it is buffered; the server keeps serving new calls."""
    srv = nns.parse_launch(f"tensor_src_grpc name=gs server=true port=0 max-recv-message-size=65536 ! {CAPS} "
                           "! tensor_sink name=sink")
    got = []
    srv.get_by_name("sink").connect("new-data", lambda b: got.append(b.memory(0).bytes()))
    srv.set_state("playing")
    port = _wait_port(srv.get_by_name("gs"))
    msgs = _messages_via_native(nns, _frames(1))
    try:
        with grpc.insecure_channel(f"127.0.0.1:{port}",
                                   options=[("grpc.max_send_message_length", -1)]) as ch:
            call = ch.stream_unary(f"/{SERVICE}/SendTensors", request_serializer=_ident, response_deserializer=_ident)
            with pytest.raises(grpc.RpcError) as e:
                call(iter([b"\x00" * (1 << 20)]), timeout=10)
            assert e.value.code() == grpc.StatusCode.RESOURCE_EXHAUSTED
            assert call(iter(msgs), timeout=10) == b""  # a normal call still works
        t0 = time.time()
        while not got and time.time() - t0 < 10:
            time.sleep(0.02)
    finally:
        srv.stop()
    assert len(got) == 1


def test_header_block_flood_closes_connection(nns):
    """A header block that keeps growing through CONTINUATION frames is cut off
    at SETTINGS_MAX_HEADER_LIST_SIZE (64 KiB): GOAWAY, connection closed."""
    import socket
    import struct

    srv = nns.parse_launch(f"tensor_src_grpc name=gs server=true port=0 ! {CAPS} ! fakesink")
    srv.set_state("playing")
    port = _wait_port(srv.get_by_name("gs"))

    def frame(ftype, flags, sid, payload):
        return struct.pack(">I", len(payload))[1:] + bytes([ftype, flags]) + struct.pack(">I", sid) + payload

    s = socket.create_connection(("127.0.0.1", port), timeout=5)
    try:
        s.sendall(b"PRI * HTTP/2.0\r\n\r\nSM\r\n\r\n" + frame(4, 0, 0, b""))
        s.sendall(frame(1, 0, 1, b"\x82"))  # HEADERS without END_HEADERS
        closed = False
        goaway = False
        buf = b""
        for _ in range(40):  # 40 x 16 KiB of CONTINUATION
            try:
                s.sendall(frame(9, 0, 1, b"\x00" * 16384))
            except OSError:
                closed = True
                break
        s.settimeout(5)
        try:
            while True:
                d = s.recv(65536)
                if not d:
                    closed = True
                    break
                buf += d
        except OSError:
            closed = True
        i = 0
        while i + 9 <= len(buf):
            ln = int.from_bytes(buf[i:i + 3], "big")
            goaway |= buf[i + 3] == 7
            i += 9 + ln
        assert closed and goaway
    finally:
        s.close()
        srv.stop()
