"""Rank-group elements (connect-type=RCCL edge / query, tensor_allgather).

On CPU the groups run with comm-backend=tcp (payload inline in the control
store), so the same element logic -- collective ordering, caps exchange,
client-id routing, EOS rounds -- is exercised without GPUs.  Ranks are
simulated in one process with explicit rank= / world-size= properties, plus
one multi-process case launched like torchrun (RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT).  The RCCL data plane is covered by
tests/test_gpu_comm.py (one GPU: single-member groups) and by the
multi-GPU bench."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

F32 = "other/tensors,format=static,num_tensors=1,dimensions=4,types=float32,framerate=0/1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    from rank_util import free_port

    return free_port()


def _rank(k, n, store, extra=""):
    return f"rank={k} world-size={n} store=127.0.0.1:{store} comm-backend=tcp comm-timeout=20000 {extra}"


def _collect(p, name="sink"):
    out = []
    p.get_by_name(name).connect("new-data", lambda b: out.append(
        (b.pts, [b.memory(i).numpy("float32").copy() for i in range(b.n_memory)])))
    return out


def _push(p, frames, src="src"):
    for i, f in enumerate(frames):
        p.get_by_name(src).push_buffer(f, pts=100 + i)
    p.get_by_name(src).end_of_stream()


def _wait_eos(p, t=30):
    msg = p.wait(t)
    assert msg and msg[0] == "eos", p.messages()


@pytest.mark.parametrize("mode", ["broadcast", "scatter"])
def test_edge_rank_group(nns, mode):
    store = _free_port()
    n = 3
    pub = nns.parse_launch(f"appsrc name=src caps={F32} ! edgesink connect-type=RCCL topic=e-{mode} "
                           f"rccl-mode={mode} {_rank(0, n, store)}")
    subs, outs = [], []
    for k in range(1, n):
        s = nns.parse_launch(f"edgesrc connect-type=RCCL topic=e-{mode} rccl-mode={mode} {_rank(k, n, store)} "
                             "! tensor_sink name=sink")
        outs.append(_collect(s))
        s.set_state("playing")
        subs.append(s)
    pub.set_state("playing")
    frames = [np.full(4, i, np.float32) for i in range(6)]
    _push(pub, frames)
    _wait_eos(pub)
    for s in subs:
        _wait_eos(s)
        s.stop()
    pub.stop()
    got = [[float(m[0][0]) for _, m in o] for o in outs]
    if mode == "broadcast":
        assert got == [[float(i) for i in range(6)]] * 2
    else:  # round-robin over the two subscribers
        assert got == [[0.0, 2.0, 4.0], [1.0, 3.0, 5.0]]
        assert [t for t, _ in outs[0]] == [100, 102, 104]


def test_query_rank_group_routes_replies(nns):
    nns.register_custom_easy("rank_triple", lambda x: [x[0] * 3],
                             [nns.TensorShape([4], np.float32)], [nns.TensorShape([4], np.float32)])
    store = _free_port()
    n = 3
    server = nns.parse_launch(f"tensor_query_serversrc connect-type=RCCL id=31 topic=q1 {_rank(0, n, store)} ! {F32} "
                              "! tensor_filter framework=custom-easy model=rank_triple "
                              "! tensor_query_serversink connect-type=RCCL id=31")
    server.set_state("playing")
    clients, outs = [], []
    for k in range(1, n):
        c = nns.parse_launch(f"appsrc name=src caps={F32} ! tensor_query_client connect-type=RCCL topic=q1 "
                             f"max-request=2 {_rank(k, n, store)} ! tensor_sink name=sink")
        outs.append(_collect(c))
        c.set_state("playing")
        clients.append(c)
    import threading
    th = [threading.Thread(target=_push, args=(c, [np.full(4, 10 * k + i, np.float32) for i in range(8)]))
          for k, c in enumerate(clients, 1)]
    [t.start() for t in th]
    [t.join() for t in th]
    for c in clients:
        _wait_eos(c)
        c.stop()
    server.stop()
    for k, o in enumerate(outs, 1):
        assert [t for t, _ in o] == [100 + i for i in range(8)]
        assert [float(m[0][0]) for _, m in o] == [3.0 * (10 * k + i) for i in range(8)]


@pytest.mark.parametrize("mode", ["concat", "stack"])
def test_allgather_rank_group(nns, mode):
    store = _free_port()
    n = 3
    caps = "other/tensors,format=static,num_tensors=1,dimensions=4:1:1:1,types=float32,framerate=0/1"
    pipes, outs = [], []
    for k in range(n):
        p = nns.parse_launch(f"appsrc name=src caps={caps} ! tensor_allgather channel=ag-{mode} mode={mode} axis=1 "
                             f"{_rank(k, n, store)} ! tensor_sink name=sink")
        outs.append(_collect(p))
        p.set_state("playing")
        pipes.append(p)
    import threading
    th = [threading.Thread(target=_push, args=(p, [np.full(4, 10 * k + i, np.float32) for i in range(4)]))
          for k, p in enumerate(pipes)]
    [t.start() for t in th]
    [t.join() for t in th]
    for p in pipes:
        _wait_eos(p)
        p.stop()
    for o in outs:
        assert len(o) == 4
        for i, (_, mems) in enumerate(o):
            if mode == "concat":
                assert [float(m[0]) for m in mems] == [float(10 * k + i) for k in range(n)]
            else:
                assert len(mems) == 1 and mems[0].shape == (12,)
                np.testing.assert_array_equal(mems[0].reshape(n, 4)[:, 0], [10 * k + i for k in range(n)])


def test_allgather_torchrun_style_processes(tmp_path):
    """Two real processes, rank / world / store from the torchrun environment."""
    script = tmp_path / "member.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {ROOT!r})
        import numpy as np
        import nnstreamer_amd as nns
        caps = "other/tensors,format=static,num_tensors=1,dimensions=2,types=float32,framerate=0/1"
        p = nns.parse_launch(f"appsrc name=src caps={{caps}} ! tensor_allgather comm-backend=tcp ! tensor_sink name=sink")
        out = []
        p.get_by_name("sink").connect("new-data", lambda b: out.append(
            [float(b.memory(i).numpy("float32")[0]) for i in range(b.n_memory)]))
        p.set_state("playing")
        r = int(os.environ["RANK"])
        for i in range(3):
            p.get_by_name("src").push_buffer(np.full(2, 100 * r + i, np.float32), pts=i)
        p.get_by_name("src").end_of_stream()
        msg = p.wait(60)
        p.stop()
        assert msg and msg[0] == "eos", p.messages()
        print("OUT", out, flush=True)
    """))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=120)[0] for p in procs]
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o
        line = [x for x in o.splitlines() if x.startswith("OUT")][0]
        assert line == "OUT [[0.0, 100.0], [1.0, 101.0], [2.0, 102.0]]", o


def test_bench_posenet_multi_two_ranks_cpu():
    """BASELINE.json config 5 through bench.py: two torchrun ranks, every rank's
    PoseNet outputs published with edgesink rccl-mode=allgather and taken back by
    one edgesrc per other camera into tensor_mux sync-mode=slowest (TCP data
    plane on CPU; RCCL on GPUs)."""
    import json
    port = _free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--cpu", "--config", "posenet_multi", "--batch", "2", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    d = json.loads(line)
    assert d["config"]["parallelism"] == "branch-dp2 + edge all-gather" and d["value"] > 0
    assert "tensor_mux name=mux sync-mode=slowest" in d["config"]["pipeline"]
    assert int(d["allgather_bytes_published_rank0"]) > 0
    assert d["mux_sets_rank0"] == 3  # warmup + steps batches, every one a full 2-camera set


@pytest.mark.parametrize("fan", ["rccl", "shm"])
def test_bench_deeplab_fan_three_ranks_cpu(fan):
    """BASELINE.json config 4 through bench.py, both fan-out transports.  rccl:
    rank 0 holds the three cameras, tensor_mux -> tensor_demux; pad 0 feeds its
    own DeepLab branch, pads 1 and 2 go to ranks 1 and 2 through edgesink
    connect-type=RCCL (two-member groups).  shm (the default): rank 0 renders
    cameras 1 and 2 into shared rings and publishes them with edgesink
    connect-type=SHM; ranks 1 and 2 subscribe and ingest their own camera."""
    import json
    port = _free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--gpus", "3", "--cpu", "--config", "deeplab_fan", "--batch", "1", "--steps", "2", "--warmup", "1",
                        "--fan-transport", fan],
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    if fan == "rccl":
        assert d["config"]["parallelism"].startswith("tensor_demux fan-out 1->3") and d["value"] > 0
        assert "tensor_demux name=d" in d["config"]["pipeline"]
    else:
        assert d["config"]["parallelism"].startswith("shared-ring fan-out 1->3") and d["value"] > 0
        assert "pool-shm=" in d["config"]["pipeline"] and "connect-type=SHM" in d["config"]["pipeline"]


def test_ini_rccl_and_hip_sections(tmp_path):
    """[rccl] timeout_ms / backend / store and [hip] keys from the ini: a rank
    group whose second member never comes fails after the ini's 400 ms
    rendezvous timeout instead of the 60 s default; nnsx-check shows the keys."""
    ini = tmp_path / "nnstreamer.ini"
    port = _free_port()
    ini.write_text(f"[rccl]\ntimeout_ms=400\nbackend=tcp\nstore=127.0.0.1:{port}\n"
                   "[hip]\npool_release_threshold=1073741824\nstream_priority=-1\n")
    script = tmp_path / "lonely.py"
    script.write_text(textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import nnstreamer_amd as nns
        caps = "other/tensors,format=static,num_tensors=1,dimensions=2,types=float32,framerate=0/1"
        p = nns.parse_launch(f"appsrc name=src caps={{caps}} ! tensor_allgather rank=0 world-size=2 ! tensor_sink")
        t0 = time.time()
        try:
            ok = p.set_state("playing")
            msg = p.wait(20)
        except Exception as e:
            ok, msg = False, ("error", "", str(e))
        print("ELAPSED", time.time() - t0, ok, msg, flush=True)
        p.stop()
    """))
    env = dict(os.environ, NNSTREAMER_CONF=str(ini), RANK="0", WORLD_SIZE="2")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=120)
    line = [x for x in r.stdout.splitlines() if x.startswith("ELAPSED")][-1]
    elapsed = float(line.split()[1])
    assert elapsed < 10, line  # not the 60 s default
    assert "False" in line or "error" in line, line
    chk = subprocess.run([os.path.join(ROOT, "bin", "nnsx-check")], env=env, capture_output=True, text=True,
                         timeout=120)
    assert "[rccl]" in chk.stdout and "timeout_ms = 400" in chk.stdout and "stream_priority = -1" in chk.stdout


def test_query_server_survives_a_crashed_client(nns, tmp_path):
    """One client rank dies without a goodbye (SIGKILL): the query server's
    any-source receive must keep serving the live client (a lost
    member link used to fail every later receive)."""
    nns.register_custom_easy("rank_double", lambda x: [x[0] * 2],
                             [nns.TensorShape([4], np.float32)], [nns.TensorShape([4], np.float32)])
    store = _free_port()
    n = 3
    server = nns.parse_launch(f"tensor_query_serversrc connect-type=RCCL id=41 topic=q2 {_rank(0, n, store)} ! {F32} "
                              "! tensor_filter framework=custom-easy model=rank_double "
                              "! tensor_query_serversink connect-type=RCCL id=41")
    server.set_state("playing")
    script = tmp_path / "crash_client.py"
    script.write_text(textwrap.dedent(f"""
        import os, signal, sys, time
        sys.path.insert(0, {ROOT!r})
        import numpy as np
        import nnstreamer_amd as nns
        c = nns.parse_launch("appsrc name=src caps={F32} ! tensor_query_client connect-type=RCCL topic=q2 "
                             "max-request=1 {_rank(2, n, store)} ! tensor_sink name=sink")
        got = []
        c.get_by_name("sink").connect("new-data", lambda b: got.append(1))
        c.set_state("playing")
        c.get_by_name("src").push_buffer(np.full(4, 7, np.float32), pts=1)
        t = time.time()
        while not got and time.time() - t < 20:
            time.sleep(0.01)
        print("replied", len(got), flush=True)
        os.kill(os.getpid(), signal.SIGKILL)
    """))
    crash = subprocess.Popen([sys.executable, str(script)], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    c = nns.parse_launch(f"appsrc name=src caps={F32} ! tensor_query_client connect-type=RCCL topic=q2 "
                         f"max-request=2 {_rank(1, n, store)} ! tensor_sink name=sink")
    out = _collect(c)
    c.set_state("playing")
    c.get_by_name("src").push_buffer(np.full(4, 0, np.float32), pts=100)  # every member joins the reply group
    crash_out, _ = crash.communicate(timeout=60)
    assert "replied 1" in crash_out and crash.returncode == -9, (crash.returncode, crash_out)
    for i in range(1, 5):
        c.get_by_name("src").push_buffer(np.full(4, i, np.float32), pts=100 + i)
    c.get_by_name("src").end_of_stream()
    _wait_eos(c)
    c.stop()
    server.stop()
    assert [float(m[0][0]) for _, m in out] == [2.0 * i for i in range(5)]


def test_edge_allgather_subscriber_stops_others_continue(tmp_path):
    """edgesink/edgesrc rccl-mode=allgather (the topic's EdgeHub): one
    subscriber of a member stops in the middle of the stream; the publisher
    and the member's other subscriber carry on and receive every frame.
    Cancellation is per waiter (comm_elements.cc EdgeHub::cancel_take /
    cancel_publish): a shared flag used to fail every later publish and take."""
    script = tmp_path / "member.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, time
        sys.path.insert(0, {ROOT!r})
        import numpy as np
        import nnstreamer_amd as nns
        rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
        caps = "other/tensors,format=static,num_tensors=1,dimensions=2,types=float32,framerate=0/1"
        edge = (f"connect-type=RCCL rccl-mode=allgather topic=stopper rank={{rank}} world-size={{world}} "
                "comm-backend=tcp comm-timeout=30000")
        others = [r for r in range(world) if r != rank]
        subs, outs = {{}}, {{}}
        for r in others:
            p = nns.parse_launch(f"edgesrc name=s {{edge}} peer-rank={{r}} ! tensor_sink name=sink")
            outs[r] = []
            p.get_by_name("sink").connect("new-data", lambda b, r=r: outs[r].append(
                float(b.memory(0).numpy("float32")[0])))
            p.set_state("playing")
            subs[r] = p
        pub = nns.parse_launch(f"appsrc name=src caps={{caps}} ! edgesink name=ag {{edge}}")
        pub.set_state("playing")
        stopped = others[0]
        for i in range(12):
            pub.get_by_name("src").push_buffer(np.full(2, 100 * rank + i, np.float32), pts=i)
            if i == 4:
                time.sleep(0.3)
                subs[stopped].stop()
        pub.get_by_name("src").end_of_stream()
        msg = pub.wait(60)
        assert msg and msg[0] == "eos", pub.messages()
        keep = others[1]
        msg = subs[keep].wait(60)
        assert msg and msg[0] == "eos", subs[keep].messages()
        subs[keep].stop()
        pub.stop()
        print("OUT", keep, outs[keep], flush=True)
    """))
    port = _free_port()
    procs = []
    for r in range(3):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="3", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=180)[0] for p in procs]
    for p, o in zip(procs, outs):
        assert p.returncode == 0, o[-3000:]
        line = [x for x in o.splitlines() if x.startswith("OUT")][0]
        _, keep, vals = line.split(" ", 2)
        assert eval(vals) == [100.0 * int(keep) + i for i in range(12)], o[-2000:]
