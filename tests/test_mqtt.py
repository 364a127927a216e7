"""mqttsink / mqttsrc over the native MQTT client and the in-process broker
(reference: tests/gstreamer_mqtt/ -- unittest_mqtt_w_helper.cc drives the
elements against a mocked paho; here a real broker runs in-process)."""
import socket
import struct
import threading
import time

import numpy as np
import pytest

F32 = "other/tensors,format=static,num_tensors=2,dimensions=4.2,types=float32.uint8,framerate=0/1"


def test_broker_wildcards_and_retained(nns):
    b = nns.MqttBroker()
    # publish a retained message with a raw socket client speaking MQTT 3.1.1
    s = socket.create_connection(("127.0.0.1", b.port))

    def pkt(t, body):
        n, enc = len(body), b""
        while True:
            d, n = n % 128, n // 128
            enc += bytes([d | (0x80 if n else 0)])
            if not n:
                break
        return bytes([t]) + enc + body

    def mstr(x):
        return struct.pack(">H", len(x)) + x

    s.sendall(pkt(0x10, mstr(b"MQTT") + b"\x04\x02\x00\x3c" + mstr(b"raw")))
    s.settimeout(5)
    connack = b""
    while len(connack) < 4:  # TCP may deliver the 4-byte CONNACK in pieces
        chunk = s.recv(4 - len(connack))
        assert chunk, "broker closed the connection"
        connack += chunk
    assert connack == b"\x20\x02\x00\x00"
    s.sendall(pkt(0x31, mstr(b"cam/0/meta") + b"hello"))  # QoS 0, retain
    time.sleep(0.1)
    # subscribe with a wildcard: the retained message is delivered at once
    s.sendall(pkt(0x82, b"\x00\x01" + mstr(b"cam/+/meta") + b"\x00"))
    data = b""
    t0 = time.time()
    while b"hello" not in data and time.time() - t0 < 5:
        data += s.recv(4096)
    assert data.startswith(b"\x90\x03\x00\x01\x00")  # SUBACK
    assert b"cam/0/meta" in data and data.endswith(b"hello")
    s.sendall(b"\xe0\x00")
    s.close()
    b.stop()


def _sub(nns, port, topic, extra=""):
    p = nns.parse_launch(f"mqttsrc name=src host=127.0.0.1 port={port} sub-topic={topic} sub-timeout=1500000 {extra} "
                         "! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda buf: out.append(
        (buf.pts, buf.memory(0).numpy("float32").copy(), buf.memory(1).numpy("uint8").copy())))
    return p, out


def test_mqtt_pubsub_tensors(nns):
    b = nns.MqttBroker()
    subs = [_sub(nns, b.port, "nnsx/test/t1") for _ in range(2)]
    for p, _ in subs:
        p.set_state("playing")
    t0 = time.time()
    while b.clients < 2 and time.time() - t0 < 5:
        time.sleep(0.01)
    time.sleep(0.2)  # subscriptions registered
    pub = nns.parse_launch(f"appsrc name=src caps={F32} ! mqttsink host=127.0.0.1 port={b.port} "
                           "pub-topic=nnsx/test/t1 mqtt-qos=1")
    pub.set_state("playing")
    frames = [(np.arange(4, dtype=np.float32) + i, np.full(2, i, np.uint8)) for i in range(5)]
    for i, (a, c) in enumerate(frames):
        pub.get_by_name("src").push_buffer([a, c], pts=1_000_000 * i)
    pub.get_by_name("src").end_of_stream()
    assert pub.wait(10)[0] == "eos"
    assert int(pub.get_by_name("mqttsink0").get_property("published")) == 5
    for p, out in subs:
        msg = p.wait(20)  # sub-timeout ends the stream
        assert msg and msg[0] == "eos", p.messages()
        p.stop()
        assert len(out) == 5
        for (pts, a, c), (ea, ec) in zip(out, frames):
            np.testing.assert_array_equal(a, ea)
            np.testing.assert_array_equal(c, ec)
        # publisher and subscriber started within the same second: re-based PTS stay ordered
        assert [x[0] for x in out] == sorted(x[0] for x in out)
    pub.stop()
    b.stop()


def test_mqtt_header_layout(nns):
    """The 1024-byte GstMQTTMessageHdr: num_mems, size_mems[16], epochs, times, caps[512]."""
    b = nns.MqttBroker()
    got = []
    ready = threading.Event()

    def recv_exact(s, n):
        buf = b""
        while len(buf) < n:
            chunk = s.recv(n - len(buf))
            if not chunk:
                break
            buf += chunk
        return buf

    def raw_sub():
        s = socket.create_connection(("127.0.0.1", b.port))
        s.sendall(b"\x10\x0f\x00\x04MQTT\x04\x02\x00\x3c\x00\x03raw")
        assert recv_exact(s, 4) == b"\x20\x02\x00\x00"
        s.sendall(b"\x82\x08\x00\x01\x00\x03hdr\x00")
        assert recv_exact(s, 5) == b"\x90\x03\x00\x01\x00"
        ready.set()
        data = b""
        t0 = time.time()
        while len(data) < 1050 and time.time() - t0 < 10:
            data += s.recv(65536)
        got.append(data)
        s.close()

    th = threading.Thread(target=raw_sub)
    th.start()
    ready.wait(5)
    pub = nns.parse_launch(f"appsrc name=src caps={F32} ! mqttsink host=127.0.0.1 port={b.port} pub-topic=hdr")
    pub.set_state("playing")
    pub.get_by_name("src").push_buffer([np.ones(4, np.float32), np.zeros(2, np.uint8)], pts=123)
    pub.get_by_name("src").end_of_stream()
    pub.wait(10)
    th.join(15)
    pub.stop()
    b.stop()
    data = got[0]
    # fixed header: PUBLISH, remaining length varint, topic "hdr"
    assert data[0] == 0x30
    i = 1
    while data[i] & 0x80:
        i += 1
    body = data[i + 1:]
    assert body[:5] == b"\x00\x03hdr"
    hdr = body[5:5 + 1024]
    num, = struct.unpack_from("<I", hdr, 0)
    sizes = struct.unpack_from("<16Q", hdr, 8)
    base, sent, dur, dts, pts = struct.unpack_from("<qqQQQ", hdr, 136)
    caps = hdr[176:176 + 512].split(b"\0")[0].decode()
    assert num == 2 and sizes[:3] == (16, 2, 0)
    assert pts == 123 and sent >= base > 0
    assert "other/tensors" in caps and "num_tensors=(int)2" in caps or "num_tensors=2" in caps
    payload = body[5 + 1024:]
    np.testing.assert_array_equal(np.frombuffer(payload[:16], np.float32), np.ones(4, np.float32))


def test_mqttsrc_requires_topic(nns):
    b = nns.MqttBroker()
    p = nns.parse_launch(f"mqttsrc port={b.port} ! fakesink")
    with pytest.raises(Exception):
        p.set_state("playing")
        msg = p.wait(5)
        assert msg is None or msg[0] == "error"
        raise RuntimeError("no topic")
    p.stop()
    b.stop()


F4 = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"


def _server(nns, broker, sid, model):
    p = nns.parse_launch(f"tensor_query_serversrc id={sid} port=0 connect-type=HYBRID dest-host=127.0.0.1 "
                         f"dest-port={broker.port} topic=hyb ! {F4} ! tensor_filter framework=custom-easy model={model} "
                         f"! tensor_query_serversink id={sid} connect-type=HYBRID")
    p.set_state("playing")
    return p


def test_query_hybrid_discovery_and_failover(nns):
    nns.register_custom_easy("hyb_x2", lambda x: [x[0] * 2], [nns.TensorShape([4], np.float32)],
                             [nns.TensorShape([4], np.float32)])
    nns.register_custom_easy("hyb_x3", lambda x: [x[0] * 3], [nns.TensorShape([4], np.float32)],
                             [nns.TensorShape([4], np.float32)])
    b = nns.MqttBroker()
    s1 = _server(nns, b, 41, "hyb_x2")
    time.sleep(0.3)
    s2 = _server(nns, b, 42, "hyb_x3")
    time.sleep(0.3)
    c = nns.parse_launch(f"appsrc name=src caps={F4} ! tensor_query_client connect-type=HYBRID dest-host=127.0.0.1 "
                         f"dest-port={b.port} topic=hyb timeout=5000 ! tensor_sink name=sink")
    out = []
    c.get_by_name("sink").connect("new-data", lambda buf: out.append(float(buf.memory(0).numpy("float32")[0])))
    c.set_state("playing")
    src = c.get_by_name("src")
    src.push_buffer(np.ones(4, np.float32), pts=0)
    t0 = time.time()
    while not out and time.time() - t0 < 10:
        time.sleep(0.01)
    first = out[0]
    assert first in (2.0, 3.0)
    # kill the server the client is talking to: the next request fails over to the other one
    (s1 if first == 2.0 else s2).stop()
    time.sleep(0.2)
    src.push_buffer(np.ones(4, np.float32), pts=1)
    src.end_of_stream()
    msg = c.wait(20)
    assert msg and msg[0] == "eos", c.messages()
    c.stop()
    assert len(out) == 2 and out[1] == (3.0 if first == 2.0 else 2.0)
    s1.stop()
    s2.stop()
    b.stop()


def test_edge_hybrid_pubsub(nns):
    b = nns.MqttBroker()
    pub = nns.parse_launch(f"appsrc name=src caps={F4} ! edgesink port=0 connect-type=HYBRID dest-host=127.0.0.1 "
                           f"dest-port={b.port} topic=cam wait-connection=1")
    pub.set_state("playing")
    time.sleep(0.3)
    sub = nns.parse_launch(f"edgesrc connect-type=HYBRID dest-host=127.0.0.1 dest-port={b.port} topic=cam "
                           "! tensor_sink name=sink")
    out = []
    sub.get_by_name("sink").connect("new-data", lambda buf: out.append(float(buf.memory(0).numpy("float32")[0])))
    sub.set_state("playing")
    for i in range(4):
        pub.get_by_name("src").push_buffer(np.full(4, i, np.float32), pts=i)
    pub.get_by_name("src").end_of_stream()
    assert pub.wait(20)[0] == "eos"
    msg = sub.wait(20)
    assert msg and msg[0] == "eos", sub.messages()
    sub.stop()
    pub.stop()
    b.stop()
    assert out == [0.0, 1.0, 2.0, 3.0]


@pytest.mark.parametrize("ctype", ["AITT", "MQTT"])
def test_edge_broker_pubsub(nns, ctype):
    """connect-type=AITT / MQTT: frames travel through the broker on the topic
    (nnstreamer-edge's broker-carried types); two subscribers each get every
    frame, one that joins late negotiates from the retained caps."""
    b = nns.MqttBroker()
    common = f"connect-type={ctype} dest-host=127.0.0.1 dest-port={b.port} topic=cam-{ctype}"
    subs, outs = [], []
    for k in range(2):
        sub = nns.parse_launch(f"edgesrc {common} ! tensor_sink name=sink")
        out = []
        sub.get_by_name("sink").connect("new-data", lambda buf, out=out: out.append(
            (float(buf.memory(0).numpy("float32")[0]), int(buf.memory(1).numpy("uint8")[1]))))
        sub.set_state("playing")
        subs.append(sub)
        outs.append(out)
    pub = nns.parse_launch(f"appsrc name=src caps={F32} ! edgesink {common}")
    pub.set_state("playing")
    src = pub.get_by_name("src")
    for i in range(3):
        src.push_buffer([np.full(4, i, np.float32), np.full(2, 10 + i, np.uint8)], pts=i)
    t0 = time.time()
    while min(len(o) for o in outs) < 3 and time.time() - t0 < 10:
        time.sleep(0.01)
    late = nns.parse_launch(f"edgesrc {common} ! tensor_sink name=sink")
    late_out = []
    late.get_by_name("sink").connect("new-data", lambda buf: late_out.append(float(buf.memory(0).numpy("float32")[0])))
    late.set_state("playing")
    for i in range(3, 5):
        src.push_buffer([np.full(4, i, np.float32), np.full(2, 10 + i, np.uint8)], pts=i)
    src.end_of_stream()
    assert pub.wait(20)[0] == "eos"
    for p in subs + [late]:
        msg = p.wait(20)
        assert msg and msg[0] == "eos", p.messages()
        p.stop()
    pub.stop()
    b.stop()
    for out in outs:
        assert out == [(float(i), 10 + i) for i in range(5)]
    assert late_out == [3.0, 4.0]


def test_query_refuses_pubsub_connect_types(nns):
    b = nns.MqttBroker()
    c = nns.parse_launch(f"appsrc name=src caps={F4} ! tensor_query_client connect-type=AITT dest-host=127.0.0.1 "
                         f"dest-port={b.port} ! tensor_sink")
    assert c.set_state("playing") is False
    msg = c.wait(10)
    assert msg[0] == "error" and "pub/sub" in msg[2], msg
    c.stop()
    b.stop()
