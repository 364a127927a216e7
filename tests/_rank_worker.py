"""One member of a rank group (comm/group.h) exercising every data-plane call:
uniform and ragged all-gather, broadcast, scatter and a send/recv ring.
Run as a child process per rank (tests/test_rank_collectives.py on CPU with the
tcp backend, tests/test_gpu_rccl_ranks.py with one GPU per rank over RCCL).

    python tests/_rank_worker.py RANK WORLD STORE_PORT DEVICE BACKEND [big]

Prints one JSON line with what it received and the group's byte counters.

`big`: frame-sized payloads instead (the real pipelines move 0.8-77 MB per
message): a 64 MB uniform all-gather, a ragged all-gather of 3-70 MB blobs
(odd sizes), a 64 MB broadcast and scatter, a send-first ring of 48 MB
messages and an all-to-all exchange of 32 MB messages in which every member
sends to every other member before receiving anything.  On one shared RCCL
comm stream the ring and the exchange are the classic cross-rank hang (each
send kernel queued ahead of the receive its peer waits for); comm::Group
carries p2p on per-direction links (comm/group.h).  Each received payload is
checked element by element against the sender's pattern (value = sender
rank * 1000 + index % 997), only a digest goes into the JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def pattern(src, n, tag=0):
    import numpy as np

    return (np.float32(src * 1000 + tag * 100) + (np.arange(n, dtype=np.int64) % 997).astype(np.float32))


def big(g, rank, world, arr, res):
    import numpy as np

    MB = 1 << 20

    def ok(m, src, n, tag=0):
        a = m.numpy("float32")
        return bool(a.size == n and np.array_equal(a, pattern(src, n, tag)))

    n64 = 64 * MB // 4
    all_, stacked = g.allgather(nns_packet([arr(pattern(rank, n64))]))
    res["big_ag"] = [ok(p.blobs[0], k, n64) for k, p in enumerate(all_)]
    if stacked is not None:
        st = stacked.numpy("float32")
        res["big_ag_stacked"] = all(np.array_equal(st[k * n64:(k + 1) * n64], pattern(k, n64)) for k in range(world))
    # ragged: 3 MB .. 70 MB, sizes not a multiple of 1 KB
    sizes = [(3 * MB + (67 * MB * k) // max(1, world - 1)) // 4 - 3 * k - 1 for k in range(world)]
    all_, _ = g.allgather(nns_packet([arr(pattern(rank, sizes[rank], 1))]))
    res["big_ag_ragged"] = [ok(p.blobs[0], k, sizes[k], 1) for k, p in enumerate(all_)]
    root = world - 1
    got = g.broadcast(root, nns_packet([arr(pattern(root, n64, 2))]) if rank == root else nns_packet())
    res["big_bcast"] = ok(got.blobs[0], root, n64, 2)
    parts = [nns_packet([arr(pattern(r, n64, 3))]) for r in range(world)] if rank == 0 else []
    mine = g.scatter(0, parts)
    res["big_scatter"] = ok(mine.blobs[0], rank, n64, 3)
    if world > 1:
        n48 = 48 * MB // 4
        nxt = (rank + 1) % world
        for k in range(2):
            g.send(nxt, nns_packet([arr(pattern(rank, n48, 4 + k))], pts=k))
        ring = []
        for _ in range(2):
            p = g.recv(120000)
            ring.append([p.src, p.pts, ok(p.blobs[0], p.src, n48, 4 + p.pts)])
        res["big_ring"] = ring
        n32 = 32 * MB // 4
        for peer in range(world):
            if peer != rank:
                g.send(peer, nns_packet([arr(pattern(rank, n32, 6))], pts=peer))
        seen = []
        for _ in range(world - 1):
            p = g.recv(120000)
            seen.append([p.src, p.pts == rank and ok(p.blobs[0], p.src, n32, 6)])
        res["big_exchange"] = sorted(seen)


def nns_packet(blobs=(), pts=-1):
    import nnstreamer_amd as nns

    return nns.Packet(list(blobs), pts=pts)


def main():
    rank, world, port, dev, backend = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]),
                                       sys.argv[5])
    mode = sys.argv[6] if len(sys.argv) > 6 else "small"
    import numpy as np

    import nnstreamer_amd as nns

    if dev >= 0:
        import torch

        torch.cuda.set_device(dev)

        def arr(v):
            return torch.as_tensor(v).cuda(dev)
    else:
        def arr(v):
            return np.asarray(v)

    g = nns.Group("test/collectives", rank, world, f"127.0.0.1:{port}", dev, backend, 60000)
    res = {"rank": rank, "backend": g.backend, "size": g.size}
    if mode in ("flush", "credit"):
        # member 1 queues 20 messages for member 0 (2.5 credit windows); member 0
        # starts receiving a second later.  flush: member 1 closes the group at
        # once -- the orderly close must deliver all of them; credit: member 1
        # stays (waits for an ack) -- member 0's receives must refresh the credit
        # member 1 used up
        import time

        if rank == 1:
            for k in range(20):
                g.send(0, nns.Packet([arr(np.full(4, k, np.float32))], pts=k))
            if mode == "credit":
                ack = g.recv(60000)
                res["ack"] = None if ack is None else ack.pts
        elif rank == 0:
            time.sleep(1.0)
            got = []
            for _ in range(20):
                p = g.recv(30000)
                got.append(None if p is None else [p.src, p.pts, float(p.blobs[0].numpy("float32")[0])])
            res["flush"] = got
            if mode == "credit":
                g.send(1, nns.Packet([arr(np.zeros(1, np.float32))], pts=99))
        del g
        print(json.dumps(res), flush=True)
        return
    if mode == "big":
        big(g, rank, world, arr, res)
        res["bytes_sent"] = g.bytes_sent
        res["bytes_received"] = g.bytes_received
        print(json.dumps(res), flush=True)
        return

    def vals(m):
        return m.numpy("float32").tolist()

    # uniform all-gather: every member sends 256 floats of its rank
    all_, stacked = g.allgather(nns.Packet([arr(np.full(256, rank, np.float32))], pts=100 + rank))
    res["ag"] = [[p.src, p.pts, vals(p.blobs[0])[0], len(vals(p.blobs[0]))] for p in all_]
    res["ag_on_device"] = [bool(p.blobs[0].on_device) for p in all_]
    res["ag_stacked"] = None if stacked is None else vals(stacked)[::256]
    # ragged all-gather: member r sends r + 1 floats of 10 r
    all_, _ = g.allgather(nns.Packet([arr(np.full(rank + 1, 10 * rank, np.float32))]))
    res["ag_ragged"] = [vals(p.blobs[0]) for p in all_]
    # broadcast from the last member
    root = world - 1
    pkt = nns.Packet([arr(np.arange(64, dtype=np.float32) + 1000)], pts=7, caps="other/tensors") \
        if rank == root else nns.Packet()
    got = g.broadcast(root, pkt)
    res["bcast"] = [got.pts, got.caps, vals(got.blobs[0])[:3]]
    # scatter from member 0: part r = 32 floats of 100 + r
    parts = [nns.Packet([arr(np.full(32, 100 + r, np.float32))], pts=r) for r in range(world)] if rank == 0 else []
    mine = g.scatter(0, parts)
    res["scatter"] = [mine.pts, vals(mine.blobs[0])[0], len(vals(mine.blobs[0]))]
    # ring: send to the next member, receive from the previous one (twice, FIFO)
    if world > 1:
        nxt = (rank + 1) % world
        for k in range(2):
            g.send(nxt, nns.Packet([arr(np.full(8, rank * 10 + k, np.float32))], pts=k))
        ring = []
        for _ in range(2):
            p = g.recv(60000)
            ring.append([p.src, p.pts, vals(p.blobs[0])[0]])
        res["ring"] = ring
    res["bytes_sent"] = g.bytes_sent
    res["bytes_received"] = g.bytes_received
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
