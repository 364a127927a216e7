"""Shared by the CPU and GPU multi-rank tests: start one tests/_rank_worker.py
child per rank (never exec'ing from this process) and check what each member
received against what every other member sent."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    """A MASTER_PORT P such that P and P + 17 are both free: comm::Group derives
    its control-plane store from MASTER_PORT + 17 (group.cc), and when that port
    is taken -- e.g. the local end of an unrelated outgoing connection -- the
    first member takes it for another member's store and the group fails."""
    for _ in range(64):
        socks = []
        try:
            s = socket.socket()
            s.bind(("127.0.0.1", 0))
            socks.append(s)
            p = s.getsockname()[1]
            if p + 17 > 65535:
                continue
            t = socket.socket()
            socks.append(t)
            t.bind(("127.0.0.1", p + 17))
            return p
        except OSError:
            continue
        finally:
            for x in socks:
                x.close()
    raise RuntimeError("no free port pair")


def run_ranks(world, devices, backend, timeout=240, mode="small"):
    port = free_port()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    procs = [subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_rank_worker.py"), str(r), str(world),
                               str(port), str(devices[r]), backend, mode], stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True, env=env) for r in range(world)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    res = []
    for rc, out in outs:
        assert rc == 0, out[-3000:]
        line = [l for l in out.splitlines() if l.startswith("{")][-1]
        res.append(json.loads(line))
    return res


def check(res, world, backend):
    for r, x in enumerate(res):
        assert x["rank"] == r and x["size"] == world and x["backend"] == backend, x
        assert x["ag"] == [[k, 100 + k, float(k), 256] for k in range(world)], x["ag"]
        if x["ag_stacked"] is not None:
            assert x["ag_stacked"] == [float(k) for k in range(world)]
        assert x["ag_ragged"] == [[10.0 * k] * (k + 1) for k in range(world)], x["ag_ragged"]
        assert x["bcast"] == [7, "other/tensors", [1000.0, 1001.0, 1002.0]], x["bcast"]
        assert x["scatter"] == [r, 100.0 + r, 32], x["scatter"]
        if world > 1:
            prv = (r - 1) % world
            assert x["ring"] == [[prv, 0, prv * 10.0], [prv, 1, prv * 10.0 + 1]], x["ring"]
            assert x["bytes_sent"] > 0 and x["bytes_received"] > 0, x


def check_big(res, world, backend):
    """Frame-sized payloads (_rank_worker.py big): every element of every
    received payload equals its sender's pattern."""
    for r, x in enumerate(res):
        assert x["rank"] == r and x["size"] == world and x["backend"] == backend, x
        assert x["big_ag"] == [True] * world, x
        assert x.get("big_ag_stacked", True), x
        assert x["big_ag_ragged"] == [True] * world, x
        assert x["big_bcast"] and x["big_scatter"], x
        if world > 1:
            prv = (r - 1) % world
            assert x["big_ring"] == [[prv, 0, True], [prv, 1, True]], x["big_ring"]
            assert x["big_exchange"] == [[k, True] for k in range(world) if k != r], x["big_exchange"]
