"""One member of a rank group (comm/group.h) exercising every data-plane call:
uniform and ragged all-gather, broadcast, scatter and a send/recv ring.
Run as a child process per rank (tests/test_rank_collectives.py on CPU with the
tcp backend, tests/test_gpu_rccl_ranks.py with one GPU per rank over RCCL).

    python tests/_rank_worker.py RANK WORLD STORE_PORT DEVICE BACKEND

Prints one JSON line with what it received and the group's byte counters."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    rank, world, port, dev, backend = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]),
                                       sys.argv[5])
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
