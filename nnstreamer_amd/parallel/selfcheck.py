"""Data-plane self-check of a rank group (csrc/comm/group.h): every
comm::Group operation the among-device elements use, on frame-sized payloads,
each received byte checked against its sender's pattern.

* all-gather, uniform (64 MB per member: one ncclAllGather, stacked output)
  and ragged (3-70 MB, odd sizes: one broadcast per root);
* broadcast (64 MB from the last member);
* scatter (64 MB parts from member 0: grouped ncclSend / ncclRecv);
* point to point: a send-first ring of 48 MB messages and an all-to-all
  exchange of 32 MB messages where every member sends to every other member
  before receiving anything (per-direction p2p links, created at group open).

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


def run(g, rank: int, world: int, arr, scale: float = 1.0) -> dict:
    """Run every operation on group `g`; `arr` turns a numpy array into a
    payload (a torch cuda tensor for device-resident blobs).  `scale` shrinks
    the payloads (CPU twins).  Returns per-operation pass flags."""
    import numpy as np

    import nnstreamer_amd as nns

    def pkt(blobs=(), pts=-1):
        return nns.Packet(list(blobs), pts=pts)

    def ok(m, src, n, tag=0):
        a = m.numpy("float32")
        return bool(a.size == n and np.array_equal(a, pattern(src, n, tag)))

    def sz(mb):
        return max(16, int(mb * MB * scale) // 4)

    res = {}
    t0 = time.perf_counter()
    n64 = sz(64)
    all_, stacked = g.allgather(pkt([arr(pattern(rank, n64))]))
    res["allgather"] = all(ok(p.blobs[0], k, n64) for k, p in enumerate(all_))
    if stacked is not None:
        st = stacked.numpy("float32")
        res["allgather_stacked"] = all(np.array_equal(st[k * n64:(k + 1) * n64], pattern(k, n64))
                                       for k in range(world))
    sizes = [max(16, (int((3 * MB + (67 * MB * k) // max(1, world - 1)) * scale)) // 4 - 3 * k - 1)
             for k in range(world)]
    all_, _ = g.allgather(pkt([arr(pattern(rank, sizes[rank], 1))]))
    res["allgather_ragged"] = all(ok(p.blobs[0], k, sizes[k], 1) for k, p in enumerate(all_))
    root = world - 1
    got = g.broadcast(root, pkt([arr(pattern(root, n64, 2))]) if rank == root else pkt())
    res["broadcast"] = ok(got.blobs[0], root, n64, 2)
    parts = [pkt([arr(pattern(r, n64, 3))]) for r in range(world)] if rank == 0 else []
    mine = g.scatter(0, parts)
    res["scatter"] = ok(mine.blobs[0], rank, n64, 3)
    if world > 1:
        # both patterns are sent before anything is received; the receives then
        # sort the messages by their pts (ring: 1000 + k, exchange: 2000 + dest)
        n48, n32 = sz(48), sz(32)
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        for k in range(2):
            g.send(nxt, pkt([arr(pattern(rank, n48, 4 + k))], pts=1000 + k))
        for peer in range(world):
            if peer != rank:
                g.send(peer, pkt([arr(pattern(rank, n32, 6))], pts=2000 + peer))
        ring, seen = [], []
        for _ in range(2 + world - 1):
            p = g.recv(120000)
            if p is None:
                break
            if 1000 <= p.pts < 1002:
                ring.append(p.src == prv and ok(p.blobs[0], p.src, n48, 4 + p.pts - 1000))
            else:
                seen.append(p.pts == 2000 + rank and ok(p.blobs[0], p.src, n32, 6))
        res["p2p_ring"] = len(ring) == 2 and all(ring)
        res["p2p_exchange"] = len(seen) == world - 1 and all(seen)
    res["seconds"] = round(time.perf_counter() - t0, 3)
    res["backend"] = g.backend
    res["size"] = g.size
    res["bytes_sent"] = g.bytes_sent
    return res
