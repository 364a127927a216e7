"""HIPIPC device-direct transport (connect-type=HIPIPC): HBM tensors cross
element/process boundaries through an exported device ring, zero-copy on the
same GPU.  Compared against the same pipelines over plain TCP."""
import os
import subprocess
import sys
import textwrap
import time

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N = 4096  # floats per tensor (16 KiB: above the inline threshold)
CAPS = f"other/tensors,format=static,num_tensors=1,dimensions={N},types=float32,framerate=0/1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _wait_port(elem, timeout=20):
    t0 = time.time()
    while time.time() - t0 < timeout:
        port = int(elem.get_property("port"))
        if port:
            return port
        time.sleep(0.01)
    raise AssertionError("server did not bind")


def _client(nns, port, frames, ctype):
    p = nns.parse_launch(f"appsrc name=src caps={CAPS} ! tensor_query_client name=qc dest-host=127.0.0.1 "
                         f"dest-port={port} connect-type={ctype} max-request=2 ! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(
        (b.memory(0).on_device, b.memory(0).numpy("float32").copy())))
    p.set_state("playing")
    for i, f in enumerate(frames):
        p.get_by_name("src").push_buffer(f, pts=i)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(60)
    stats = p.get_by_name("qc").get_property("ipc-blobs")
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    return out, stats


def _server_desc(port=0):
    return (f"tensor_query_serversrc name=qs port={port} ! {CAPS} "
            "! tensor_transform mode=arithmetic option=mul:2 ! tensor_query_serversink")


@pytest.mark.parametrize("ctype", ["TCP", "HIPIPC"])
def test_query_device_tensors_in_process(nns, ctype):
    server = nns.parse_launch(_server_desc())
    server.set_state("playing")
    port = _wait_port(server.get_by_name("qs"))
    frames = [torch.arange(N, dtype=torch.float32, device="cuda") + i for i in range(12)]
    out, stats = _client(nns, port, frames, ctype)
    server.stop()
    assert len(out) == 12
    for (_, y), x in zip(out, frames):
        np.testing.assert_array_equal(y, 2 * x.cpu().numpy())
    sent, recv = (int(v) for v in stats.split(":"))
    if ctype == "HIPIPC":
        # the first request goes as bytes while the handshake completes
        assert sent >= 10 and recv >= 10, stats
        assert all(d for d, _ in out[2:])
    else:
        assert sent == recv == 0


def test_query_hipipc_across_processes(nns, tmp_path):
    script = tmp_path / "server.py"
    script.write_text(textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import nnstreamer_amd as nns
        p = nns.parse_launch({_server_desc()!r})
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
        frames = [torch.full((N,), float(i), device="cuda") for i in range(16)]
        out, stats = _client(nns, port, frames, "HIPIPC")
        assert [float(y[0]) for _, y in out] == [2.0 * i for i in range(16)]
        sent, recv = (int(v) for v in stats.split(":"))
        assert sent >= 14 and recv >= 14, stats
    finally:
        proc.stdin.write("\n")
        proc.stdin.flush()
        proc.wait(timeout=60)


def test_edge_hipipc_pubsub(nns):
    pub = nns.parse_launch(f"appsrc name=src caps={CAPS} ! edgesink name=es port=0 wait-connection=1")
    pub.set_state("playing")
    port = _wait_port(pub.get_by_name("es"))
    sub = nns.parse_launch(f"edgesrc name=er dest-host=127.0.0.1 dest-port={port} connect-type=HIPIPC "
                           "! tensor_sink name=sink")
    got = []
    sub.get_by_name("sink").connect("new-data", lambda b: got.append(b.memory(0).numpy("float32")[0].item()))
    sub.set_state("playing")
    time.sleep(0.5)  # let the subscriber's IPC handshake land before publishing
    for i in range(8):
        pub.get_by_name("src").push_buffer(torch.full((N,), float(i), device="cuda"), pts=i)
    pub.get_by_name("src").end_of_stream()
    assert pub.wait(30)[0] == "eos"
    msg = sub.wait(30)
    n_ipc = int(sub.get_by_name("er").get_property("ipc-blobs"))
    sub.stop()
    pub.stop()
    assert msg and msg[0] == "eos", sub.messages()
    assert got == [float(i) for i in range(8)]
    assert n_ipc == 8


def test_allgather_rccl_single_member(nns):
    """connect-type RCCL plumbing on one GPU: an RCCL communicator of one rank
    (ncclCommInitRank + comm stream), tensors stay in HBM end to end."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    p = nns.parse_launch(
        f"appsrc name=src caps={CAPS} ! tensor_transform mode=arithmetic option=mul:2 device=0 "
        f"! tensor_allgather name=ag rank=0 world-size=1 device=0 comm-backend=rccl store=127.0.0.1:{port} mode=stack axis=1 "
        "! tensor_sink name=sink")
    out = []
    p.get_by_name("sink").connect("new-data", lambda b: out.append(
        (b.memory(0).on_device, b.memory(0).numpy("float32").copy())))
    p.set_state("playing")
    frames = [np.arange(N, dtype=np.float32) + i for i in range(3)]
    for i, f in enumerate(frames):
        p.get_by_name("src").push_buffer(f, pts=i)
    p.get_by_name("src").end_of_stream()
    msg = p.wait(60)
    p.stop()
    assert msg and msg[0] == "eos", p.messages()
    assert len(out) == 3
    for (on_dev, y), x in zip(out, frames):
        assert on_dev
        np.testing.assert_array_equal(y, 2 * x)


def _port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("mb", [1, 64])
def test_group_of_one_forced_rccl_runs_every_call(nns, mb):
    """backend=rccl on a group of one runs the real RCCL calls on one GPU: the
    one-rank ncclAllGather (a copy into the gathered buffer), ncclBroadcast and
    a grouped ncclSend/ncclRecv to itself for p2p (comm/group.cc self_copy) --
    the received blobs are fresh device buffers holding the sent bytes."""
    n = mb * (1 << 20) // 4
    g = nns.Group(f"test/one-{mb}", 0, 1, f"127.0.0.1:{_port()}", 0, "rccl", 60000)
    assert g.backend == "rccl" and g.size == 1
    x = torch.arange(n, dtype=torch.float32, device="cuda") % 997 + 1
    all_, stacked = g.allgather(nns.Packet([x], pts=5))
    assert len(all_) == 1 and all_[0].blobs[0].on_device
    assert all_[0].blobs[0].data_ptr != x.data_ptr()  # the gathered copy, not the input
    assert np.array_equal(all_[0].blobs[0].numpy("float32"), x.cpu().numpy())
    assert stacked is not None and np.array_equal(stacked.numpy("float32"), x.cpu().numpy())
    got = g.broadcast(0, nns.Packet([x], pts=6))
    assert np.array_equal(got.blobs[0].numpy("float32"), x.cpu().numpy())
    g.send(0, nns.Packet([x, x[: n // 3]], pts=7))
    p = g.recv(60000)
    assert p is not None and p.pts == 7 and len(p.blobs) == 2
    assert all(b.on_device for b in p.blobs) and p.blobs[0].data_ptr != x.data_ptr()
    assert np.array_equal(p.blobs[0].numpy("float32"), x.cpu().numpy())
    assert np.array_equal(p.blobs[1].numpy("float32"), x[: n // 3].cpu().numpy())
    assert g.bytes_sent >= 4 * (n + n // 3) and g.bytes_received >= 4 * (n + n // 3)
