"""Data-plane self-check of a rank group (csrc/comm/group.h): every
comm::Group operation the among-device elements use, on frame-sized payloads,
each received byte checked against its sender's pattern.

* all-gather, uniform (64 MB per member: one ncclAllGather, stacked output)
  and ragged (3-70 MB, odd sizes: one broadcast per root);
* broadcast (64 MB from the last member);
* scatter (64 MB parts from member 0: grouped ncclSend / ncclRecv);
* point to point: a send-first ring of 48 MB messages and an all-to-all
  exchange of 32 MB messages where every member sends to every other member
  before receiving anything (deadlock-free by construction: every operation
  runs in the group's matched rounds, csrc/comm/group.h).

Every operation is checked on its own: an operation that raises (a member
missing, a timeout, an aborted communicator) is recorded as failed with its
error in `errors`, and the next one still runs, so a broken data plane costs
the caller a bounded time and a `False`, never a hang.  Fault injection for
the CPU twin: NNSX_SELFCHECK_FAULT="<rank>:<op>" makes that rank skip the
named operation (allgather, allgather_ragged, broadcast, scatter, p2p).

Used by bench.py before its timed run when WORLD_SIZE > 1 (`rccl_selfcheck`
in its JSON) and by tests/_rank_worker.py.  Reference fan-out / fan-in points
these collectives carry: gsttensor_demux.c:469-556, edge_sink.c:305-345,
tensor_query_client.c:657-746, nnstreamer_plugin_api_impl.c:266-441.
"""
from __future__ import annotations

import time

MB = 1 << 20


def pattern(src, n, tag=0):
    import numpy as np

    return np.float32(src * 1000 + tag * 100) + (np.arange(n, dtype=np.int64) % 997).astype(np.float32)


def run(g, rank: int, world: int, arr, scale: float = 1.0, recv_timeout_ms: int = 120000) -> dict:
    """Run every operation on group `g`; `arr` turns a numpy array into a
    payload (a torch cuda tensor for device-resident blobs).  `scale` shrinks
    the payloads (CPU twins).  Returns per-operation pass flags and, for the
    operations that raised, their errors."""
    import os

    import numpy as np

    import nnstreamer_amd as nns

    fault = os.environ.get("NNSX_SELFCHECK_FAULT", "")
    skip = fault.split(":", 1)[1] if fault.startswith(f"{rank}:") else ""

    def pkt(blobs=(), pts=-1):
        return nns.Packet(list(blobs), pts=pts)

    def ok(m, src, n, tag=0):
        a = m.numpy("float32")
        return bool(a.size == n and np.array_equal(a, pattern(src, n, tag)))

    def sz(mb):
        return max(16, int(mb * MB * scale) // 4)

    res, errors = {}, {}

    def step(name, fn):
        if skip == name:
            res[name] = False
            errors[name] = "skipped (NNSX_SELFCHECK_FAULT)"
            return
        try:
            fn()
        except Exception as e:  # noqa: BLE001 -- a failed operation is a result, not a crash
            res[name] = False
            errors[name] = str(e)[:300]

    t0 = time.perf_counter()
    n64 = sz(64)

    def ag():
        all_, stacked = g.allgather(pkt([arr(pattern(rank, n64))]))
        res["allgather"] = all(ok(p.blobs[0], k, n64) for k, p in enumerate(all_))
        if stacked is not None:
            st = stacked.numpy("float32")
            res["allgather_stacked"] = all(np.array_equal(st[k * n64:(k + 1) * n64], pattern(k, n64))
                                           for k in range(world))

    def ag_ragged():
        sizes = [max(16, (int((3 * MB + (67 * MB * k) // max(1, world - 1)) * scale)) // 4 - 3 * k - 1)
                 for k in range(world)]
        all_, _ = g.allgather(pkt([arr(pattern(rank, sizes[rank], 1))]))
        res["allgather_ragged"] = all(ok(p.blobs[0], k, sizes[k], 1) for k, p in enumerate(all_))

    def bcast():
        root = world - 1
        got = g.broadcast(root, pkt([arr(pattern(root, n64, 2))]) if rank == root else pkt())
        res["broadcast"] = ok(got.blobs[0], root, n64, 2)

    def scat():
        parts = [pkt([arr(pattern(r, n64, 3))]) for r in range(world)] if rank == 0 else []
        mine = g.scatter(0, parts)
        res["scatter"] = ok(mine.blobs[0], rank, n64, 3)

    def p2p():
        # both patterns are sent before anything is received; the receives then
        # sort the messages by their pts (ring: 1000 + k, exchange: 2000 + dest)
        n48, n32 = sz(48), sz(32)
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        res["p2p_ring"] = res["p2p_exchange"] = False
        for k in range(2):
            g.send(nxt, pkt([arr(pattern(rank, n48, 4 + k))], pts=1000 + k))
        for peer in range(world):
            if peer != rank:
                g.send(peer, pkt([arr(pattern(rank, n32, 6))], pts=2000 + peer))
        ring, seen = [], []
        for _ in range(2 + world - 1):
            p = g.recv(recv_timeout_ms)
            if p is None:
                errors["p2p"] = f"a message did not arrive within {recv_timeout_ms} ms"
                break
            if 1000 <= p.pts < 1002:
                ring.append(p.src == prv and ok(p.blobs[0], p.src, n48, 4 + p.pts - 1000))
            else:
                seen.append(p.pts == 2000 + rank and ok(p.blobs[0], p.src, n32, 6))
        res["p2p_ring"] = len(ring) == 2 and all(ring)
        res["p2p_exchange"] = len(seen) == world - 1 and all(seen)

    step("allgather", ag)
    step("allgather_ragged", ag_ragged)
    step("broadcast", bcast)
    step("scatter", scat)
    if world > 1:
        step("p2p", p2p)
        if skip == "p2p":
            res["p2p_ring"] = res["p2p_exchange"] = False
        res.pop("p2p", None)
    res["seconds"] = round(time.perf_counter() - t0, 3)
    res["backend"] = g.backend
    res["size"] = g.size
    res["bytes_sent"] = g.bytes_sent
    if errors:
        res["errors"] = errors
    return res
